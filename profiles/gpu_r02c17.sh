#!/bin/bash
# routed step: the global order as arrays, the all-gather payload from numpy
set -o pipefail
O=gpurun_out/r02c17; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_routed_threads.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2; do timeout -k 10 300 python3 -u bench.py --routed --steps 6 --no-cpu > $O/routed_$r.json 2> $O/routed_$r.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/routed_$r.json | head -1) $(grep -o '"phase_ms_one_unpipelined_step_max_over_ranks": {[^}]*}' $O/routed_$r.json)"; done
