#!/bin/bash
# Round 3: fp_commit timing variants on config 2 (non-temporal row stores; 4 / 6 waves
# per SIMD), alternating fresh processes on one box, cached workload; then a kernel
# trace of the default bench command (config 2 + create_accounts of 1M accounts).
OUT=gpurun_out/r03h
mkdir -p "$OUT"
export TB_BENCH_CACHE=/tmp/tbcache
ARGS="--steps 5 --warmup 2 --no-cpu --no-queries --no-host"
REPS=1 timeout -k 10 900 python3 profiles/variants.py base ntrows w4 w6 base ntrows w4 w6 -- $ARGS > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c2 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-queries --no-host > "$OUT/c2_prof.json" 2> "$OUT/c2_prof.err" || exit $?
find "$OUT/prof" -name "*stats.csv"
