#!/bin/bash
# GPU suite on the tree, then config 3: the product (group resolution in its own
# workgroups, per-digit histogram scan) against build/var_nosplit and TBGPU_SORT_ONE_SCAN=1
set -o pipefail
O=gpurun_out/${TAG:-r04sa}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_prod.$r.json 2> /dev/null || exit 2
  TBGPU_LIB=tigerbeetle_amd/build/var_nosplit/libtbgpu.so timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_nosplit.$r.json 2> /dev/null || exit 3
  TBGPU_SORT_ONE_SCAN=1 timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_onescan.$r.json 2> /dev/null || exit 4
done
