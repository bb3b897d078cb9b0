#!/bin/bash
set -o pipefail
O=gpurun_out/r02k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
for cb in 16 30 60; do
TBGPU_CHUNK_BATCHES=$cb timeout -k 10 300 python -u bench.py --config 3 --no-queries --no-host --no-cpu > $O/bench_c3_$cb.json 2> $O/bench_c3_$cb.err; echo "c3 cb=$cb rc=$? $(grep -o '"value": [0-9.]*' $O/bench_c3_$cb.json) $(grep -o '"fixed_point_passes": [0-9]*' $O/bench_c3_$cb.json)"
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt3 -o kt --output-format csv -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/kt3.log 2>&1; echo "kt3 rc=$?"
timeout -k 10 600 python -u bench.py --config 5 --no-queries > $O/bench_c5.json 2> $O/bench_c5.err; echo "c5 rc=$?"; cat $O/bench_c5.json
