#!/bin/bash
# config 3: the evaluation launch's workgroup size, 256 (product) against 128 and 512 (build/var_ev*)
set -o pipefail
O=gpurun_out/${TAG:-r04ev}; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_prod.$r.json 2> /dev/null || exit 1
  TBGPU_LIB=tigerbeetle_amd/build/var_ev128/libtbgpu.so timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_ev128.$r.json 2> /dev/null || exit 2
  TBGPU_LIB=tigerbeetle_amd/build/var_ev512/libtbgpu.so timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_ev512.$r.json 2> /dev/null || exit 3
done
