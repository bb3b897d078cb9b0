#!/bin/bash
# config 3: general-path chunk size sweep on the current code (TBGPU_CHUNK_BATCHES)
set -o pipefail
O=gpurun_out/r02c27; mkdir -p $O
export TMPDIR=/tmp
for B in 20 30 15 24 20 12; do
  TBGPU_CHUNK_BATCHES=$B timeout -k 10 200 python3 -u bench.py --config 3 --steps 4 --no-queries --no-cpu --no-host > $O/c3_$B.json 2> $O/c3_$B.err; echo "chunk=$B rc=$? $(grep -o '"value": [0-9.]*' $O/c3_$B.json | head -1) $(grep -o '"fixed_point_passes": [0-9]*' $O/c3_$B.json)"
done
