#!/bin/bash
# Round 3: the whole -m gpu suite on the fixes (walk error word, block-aggregated list
# and group cursors), then config 3 again.
OUT=gpurun_out/r03e
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.txt"; cat gpurun_out/tbgpu_fatal.log 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-queries --no-host > "$OUT/c3.json" 2> "$OUT/c3.err" || exit $?
python3 profiles/r03/line.py "$OUT/c3.json"
