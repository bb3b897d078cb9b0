#!/bin/bash
# GPU suite on the tree, then config 3: the product (the headroom scan with two sides per
# thread in 256-thread workgroups) against build/var_nf1 (one side per thread, 512 threads)
set -o pipefail
O=gpurun_out/${TAG:-r04nf}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.txt 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_prod.$r.json 2> /dev/null || exit 2
  TBGPU_LIB=tigerbeetle_amd/build/var_nf1/libtbgpu.so timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_nf1.$r.json 2> /dev/null || exit 3
done
