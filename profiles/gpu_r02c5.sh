#!/bin/bash
# config 3: per-pass change counts (TBGPU_TRACE_PASSES) for one step
set -o pipefail
O=gpurun_out/r02c5; mkdir -p $O
export TMPDIR=/tmp
TBGPU_TRACE_PASSES=1 timeout -k 10 300 python3 -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu --no-queries --no-host > $O/c3.json 2> $O/c3_trace.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/c3.json)"
