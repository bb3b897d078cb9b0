#!/bin/bash
set -o pipefail
O=gpurun_out/r02u; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --routed --steps 2 > $O/kt.log 2>&1; echo "kt rc=$?"
