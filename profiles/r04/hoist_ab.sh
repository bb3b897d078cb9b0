#!/bin/bash
# config 3: the scans' window checks issued before the group resolution (product) against
# the previous order (build/var_nohoist), and sparse-pass thresholds n/8, n/16
set -o pipefail
O=gpurun_out/${TAG:-r04ho}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_hoist.$r.json 2> $O/c3_hoist.$r.err || exit 1
  TBGPU_LIB=tigerbeetle_amd/build/var_nohoist/libtbgpu.so timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_nohoist.$r.json 2> $O/c3_nohoist.$r.err || exit 2
  TBGPU_SPARSE_SHIFT=3 timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_s3.$r.json 2> $O/c3_s3.$r.err || exit 3
done
