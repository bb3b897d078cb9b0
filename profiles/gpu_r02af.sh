#!/bin/bash
# incremental passes: general-path parity, then config 3 timing (incremental vs full passes)
set -o pipefail
O=gpurun_out/r02af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_general.py tests/test_gpu_golden.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u bench.py --config 3 --no-queries --no-host --cpu-seconds 2 --verify > $O/c3.json 2> $O/c3.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/c3.json | head -1)"
TBGPU_FULL_PASSES=1 timeout -k 10 300 python3 -u bench.py --config 3 --no-queries --no-host --no-cpu > $O/c3full.json 2> $O/c3full.err; echo "c3full rc=$? $(grep -o '"value": [0-9.]*' $O/c3full.json | head -1)"
