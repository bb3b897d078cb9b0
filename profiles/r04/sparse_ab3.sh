#!/bin/bash
# config 3 on the round's last tree: the sparse-pass threshold with 30-batch chunks: n/16, n/8 (default), n/4
set -o pipefail
O=gpurun_out/${TAG:-r04sp3}; mkdir -p $O
for r in 1 2 3; do
  for v in 4 3 2; do
    TBGPU_SPARSE_SHIFT=$v timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_s$v.$r.json 2> /dev/null || exit 1
  done
done
