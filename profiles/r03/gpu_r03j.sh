#!/bin/bash
# Round 3: zeroed-buffer create_accounts probe (profiles/r03/acc_copy_probe.py), then the
# relay-chain test alone.
OUT=gpurun_out/r03j
mkdir -p "$OUT"
timeout -k 10 300 python3 -u profiles/r03/acc_copy_probe.py > "$OUT/probe.txt" 2>&1
rc=$?; cat "$OUT/probe.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_gpu_general.py::test_adversarial_relay_chain" > "$OUT/relay.txt" 2>&1
rc=$?; tail -5 "$OUT/relay.txt"; exit $rc
