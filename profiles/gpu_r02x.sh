#!/bin/bash
set -o pipefail
O=gpurun_out/r02x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config 3 --no-queries --no-host --no-cpu > $O/c3.json 2> $O/c3.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/c3.json) $(grep -o '"fixed_point_passes": [0-9]*' $O/c3.json)"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/kt.log 2>&1; echo "kt rc=$?"
