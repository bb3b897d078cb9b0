#!/bin/bash
# general path: one copy per chunk for the batch tables, one per pass group for counters + ring
set -o pipefail
O=gpurun_out/r02c12; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_general.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_checkpoint.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2; do timeout -k 10 300 python3 -u bench.py --config 3 --steps 4 --no-queries --no-cpu --no-host > $O/c3_$r.json 2> $O/c3_$r.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/c3_$r.json | head -1)"; done
