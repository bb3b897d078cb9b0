#!/bin/bash
set -o pipefail
O=gpurun_out/r02y; mkdir -p $O
export TMPDIR=/tmp
TBGPU_EVAL_PROBE=1 timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 0 --no-queries --no-host --no-cpu > $O/c3.json 2> $O/c3.err; echo "rc=$?"; grep "probe" $O/c3.err | head -24
