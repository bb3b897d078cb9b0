#!/bin/bash
set -o pipefail
O=gpurun_out/r02o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "blocked or dense or config4" > $O/t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config 4 --no-queries --no-host --no-cpu > $O/c4.json 2> $O/c4.err; echo "c4 rc=$? $(grep -o '"value": [0-9.]*' $O/c4.json) $(grep -o '"frac": [0-9.]*' $O/c4.json | head -1)"
timeout -k 10 300 python -u bench.py --no-queries --no-host --no-cpu > $O/c2.json 2> $O/c2.err; echo "c2 rc=$? $(grep -o '"value": [0-9.]*' $O/c2.json) $(grep -o '"frac": [0-9.]*' $O/c2.json | head -1)"
