#!/bin/bash
set -o pipefail
O=gpurun_out/r02l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_general.py tests/test_gpu_parity.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config 3 --no-queries --no-host --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_c3.json) $(grep -o '"fixed_point_passes": [0-9]*' $O/bench_c3.json)"
timeout -k 10 600 python -u bench.py --config 5 --no-queries > $O/bench_c5.json 2> $O/bench_c5.err; echo "c5 rc=$?"; cat $O/bench_c5.json
