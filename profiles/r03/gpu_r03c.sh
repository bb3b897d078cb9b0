#!/bin/bash
# Round 3, session 2: config 3 (general path) on the current code -- the bench line,
# per-pass change counts and a kernel trace -- and the memory-side atomics micro-benchmark.
OUT=gpurun_out/r03c
mkdir -p "$OUT"
hipcc --offload-arch=gfx950 -O3 profiles/micro/atomics_density.hip -o profiles/micro/atomics_density || exit 1
timeout -k 10 60 ./profiles/micro/atomics_density > "$OUT/atomics_density.txt" 2>&1 || exit $?
cat "$OUT/atomics_density.txt"
timeout -k 10 300 python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-queries --no-host > "$OUT/c3.json" 2> "$OUT/c3.err" || exit $?
python3 profiles/r03/line.py "$OUT/c3.json"
timeout -k 10 300 env TBGPU_TRACE_PASSES=1 python3 bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-queries --no-host > "$OUT/c3_trace.json" 2> "$OUT/c3_trace.err" || exit $?
grep -c "pass" "$OUT/c3_trace.err"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c3 -- python3 bench.py --config 3 --steps 1 --warmup 1 --no-cpu --no-queries --no-host > "$OUT/c3_prof.json" 2> "$OUT/c3_prof.err" || exit $?
find "$OUT/prof" -name "*kernel_stats.csv" | head -3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 || { tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 120 python3 __graft_entry__.py smoke > "$OUT/smoke.txt" 2>&1 || exit $?
cat "$OUT/smoke.txt"
