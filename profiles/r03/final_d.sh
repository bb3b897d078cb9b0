#!/bin/bash
# Round 3: the -m gpu suite and smoke on the final engine (quick check).
OUT=${1:-gpurun_out/r03_final}
mkdir -p "$OUT"
rm -f gpurun_out/tbgpu_fatal.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.out" 2> "$OUT/gpu_tests.err"
rc=$?
tail -2 "$OUT/gpu_tests.out"; grep "^FAILED" "$OUT/gpu_tests.out"
{ [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || { cat gpurun_out/tbgpu_fatal.log 2>/dev/null; exit $rc; }
timeout -k 10 180 python3 -u __graft_entry__.py smoke > "$OUT/smoke.out" 2>&1 && cat "$OUT/smoke.out"
