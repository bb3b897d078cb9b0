#!/bin/bash
set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err; echo "rc=$?"; cat $O/driver_cmd.json | head -c 2500
