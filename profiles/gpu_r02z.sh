#!/bin/bash
set -o pipefail
O=gpurun_out/r02z; mkdir -p $O
export TMPDIR=/tmp
for cb in 20 30 40; do
TBGPU_CHUNK_BATCHES=$cb timeout -k 10 300 python -u bench.py --config 3 --no-queries --no-host --no-cpu > $O/c3_$cb.json 2> $O/c3_$cb.err; echo "cb=$cb rc=$? $(grep -o '"value": [0-9.]*' $O/c3_$cb.json) $(grep -o '"fixed_point_passes": [0-9]*' $O/c3_$cb.json)"
done
