#!/bin/bash
set -o pipefail
O=gpurun_out/r02ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_routed_threads.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --routed --steps 4 > $O/routed1.json 2> $O/routed1.err; echo "routed1 rc=$?"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"phase_ms_one_unpipelined_step_max_over_ranks": {[^}]*}' $O/routed1.json; tail -2 $O/routed1.err
