#!/bin/bash
# config 3: the even cut at 32 (two chunks of 30 per call) against one chunk of 60 and 4 of 15
set -o pipefail
O=gpurun_out/${TAG:-r04cb}; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_prod.$r.json 2> /dev/null || exit 1
  TBGPU_CHUNK_BATCHES=60 timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_b60.$r.json 2> /dev/null || exit 2
  TBGPU_CHUNK_BATCHES=15 timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_b15.$r.json 2> /dev/null || exit 3
done
