#!/bin/bash
# config 3: chunks cut evenly at a limit of 32 batches (product: two of 30 per 60-batch call)
# against the even cut at 20 (three of 20), plus the general GPU tests
set -o pipefail
O=gpurun_out/${TAG:-r04ca}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.txt 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_prod.$r.json 2> /dev/null || exit 2
  TBGPU_CHUNK_BATCHES=20 timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_b20.$r.json 2> /dev/null || exit 3
  TBGPU_CHUNK_BATCHES=24 timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_b24.$r.json 2> /dev/null || exit 4
done
