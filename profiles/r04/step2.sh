#!/bin/bash
# round-4 iteration run: the GPU suite, config-3 timing, the chunk-size sweep, a trace
set -o pipefail
O=gpurun_out/${TAG:-r04s2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1 || exit 1
B="python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host"
for k in 1 2; do timeout -k 10 300 $B > $O/c3_$k.json 2> $O/c3_$k.err || exit 2; done
for cb in 12 16 28 40; do TBGPU_CHUNK_BATCHES=$cb timeout -k 10 300 $B > $O/c3_cb$cb.json 2> $O/c3_cb$cb.err || exit 3; done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- \
  python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host > $O/kt.log 2>&1 || exit 4
