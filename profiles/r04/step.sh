#!/bin/bash
# round-4 iteration run: parity of the general path, then config-3 timing (+ kernel trace)
set -o pipefail
O=gpurun_out/${TAG:-r04s}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_general.py tests/test_gpu_parity.py tests/test_gpu_prefetch.py tests/test_gpu_fuzz.py > $O/tests.txt 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host \
    > $O/c3_$k.json 2> $O/c3_$k.err || exit 2
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- \
  python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host > $O/kt.log 2>&1 || exit 3
TBGPU_TRACE_PASSES=1 timeout -k 10 200 python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-queries --no-subconfigs --no-host \
  > $O/trace.json 2> $O/trace.err || exit 4
