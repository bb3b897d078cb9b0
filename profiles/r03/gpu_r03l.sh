#!/bin/bash
# Round 3: the dense-directory parity failure: its workload on both paths (alone), with
# dirty tracking off, and after the full-size config-2 test in one process.
OUT=gpurun_out/r03l
mkdir -p "$OUT"
timeout -k 10 300 python3 -u profiles/r03/dense_probe.py 4 > "$OUT/probe.txt" 2>&1
rc=$?; cat "$OUT/probe.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env TBGPU_NO_INCR=1 python3 -u profiles/r03/dense_probe.py 3 > "$OUT/probe_noincr.txt" 2>&1
rc=$?; cat "$OUT/probe_noincr.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py \
  "tests/test_gpu_parity.py::test_dense_directory_boundaries" "tests/test_gpu_general.py::test_adversarial_relay_chain" > "$OUT/after_fullsize.txt" 2>&1
rc=$?; tail -4 "$OUT/after_fullsize.txt"; grep -m4 "^FAILED\|^E  " "$OUT/after_fullsize.txt"
exit 0
