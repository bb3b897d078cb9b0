#!/bin/bash
# router: 4-byte packed wire format, split route / exchange phases, pipelined stream
set -o pipefail
O=gpurun_out/r02c3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_routed_threads.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 -u bench.py --routed --steps 6 --no-cpu > $O/routed.json 2> $O/routed.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/routed.json)"
timeout -k 10 400 python3 -u bench.py --routed --pipelined --steps 6 --no-cpu > $O/routed_pipe.json 2> $O/routed_pipe.err; echo "pipelined rc=$? $(grep -o '"value": [0-9.]*' $O/routed_pipe.json)"
