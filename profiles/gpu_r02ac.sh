#!/bin/bash
set -o pipefail
O=gpurun_out/r02ac; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py --no-queries --no-cpu > $O/c2.json 2> $O/c2.err; echo "c2 rc=$?"; grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"host_path": {.*}}' $O/c2.json | head -4
timeout -k 10 400 python -u bench.py --routed --steps 4 --no-cpu > $O/routed1.json 2> $O/routed1.err; echo "routed1 rc=$? $(grep -o '"value": [0-9.]*' $O/routed1.json)"
