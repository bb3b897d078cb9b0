#!/bin/bash
# Round 2: the general path with device-side pass control: GPU tests, then the config-3 bench.
set -o pipefail
O=gpurun_out/r02c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|relay" $O/gpu_tests.log | tail -8
[ $rc -eq 0 ] || exit 1
TBGPU_TRACE_PASSES=1 timeout -k 10 300 python -u bench.py --config 3 --no-queries --no-host > $O/bench_c3.json 2> $O/bench_c3.err; echo "c3 rc=$?"; cat $O/bench_c3.json
grep "pass" $O/bench_c3.err | tail -40
