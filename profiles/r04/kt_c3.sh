#!/bin/bash
# config 3 kernel trace only (the per-pass timeline of the last tree)
set -o pipefail
O=gpurun_out/${TAG:-r04kt}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host > "$O/kt.log" 2>&1 || exit 1
