#!/bin/bash
# router: packed wire format, LDS-staged scatter, async commit-timestamp advance
set -o pipefail
O=gpurun_out/r02c1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_routed_threads.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 -u bench.py --routed --steps 4 --no-cpu > $O/routed.json 2> $O/routed.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/routed.json)"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --routed --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/kt.log 2>&1; echo "kt rc=$?"
