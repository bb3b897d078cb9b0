#!/bin/bash
# Round 3, first combined GPU call: the whole -m gpu suite, the drift A/B, config 3 sweep.
OUT=gpurun_out/r03a
mkdir -p "$OUT"
timeout -k 10 60 ./profiles/micro/atomics_density > "$OUT/atomics_density.txt" 2>&1; cat "$OUT/atomics_density.txt"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.txt"
[ $rc -eq 0 ] || exit $rc
bash profiles/r03/diag_drift.sh "$OUT/drift" || exit 1
bash profiles/r03/diag_config3.sh "$OUT/c3"
