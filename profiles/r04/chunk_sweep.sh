#!/bin/bash
# config 3 chunk sizes with sparse passes (TBGPU_CHUNK_BATCHES)
set -o pipefail
O=gpurun_out/${TAG:-r04cs}; mkdir -p $O
for b in 20 28 40 20 28 40; do
  TBGPU_CHUNK_BATCHES=$b timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_b$b.$RANDOM.json 2> /dev/null || exit 1
done
