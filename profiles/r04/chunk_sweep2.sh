#!/bin/bash
# config 3 chunk sizes on the round's last tree (TBGPU_CHUNK_BATCHES), alternating
set -o pipefail
O=gpurun_out/${TAG:-r04cs2}; mkdir -p $O
for r in 1 2 3; do
  for b in 16 20 24 32 40; do
    TBGPU_CHUNK_BATCHES=$b timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_b$b.$r.json 2> /dev/null || exit 1
  done
done
