#!/bin/bash
# config 3 kernel trace after the gated epilogue
set -o pipefail
O=gpurun_out/r02c21; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/kt.log 2>&1; echo "kt rc=$?"
