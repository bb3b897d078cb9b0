#!/bin/bash
# drop-in call latency A/B on one box: spin-waited small calls vs the blocking wait, alternating
set -o pipefail
O=gpurun_out/${TAG:-r04h2}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_index.py tests/test_gpu_prefetch.py tests/test_gpu_general.py tests/test_gpu_checkpoint.py \
  tests/test_gpu_parity.py > $O/tests.txt 2>&1 || exit 1
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-queries --no-subconfigs"
for k in 1 2; do
  timeout -k 10 300 $B > $O/spin_$k.json 2> $O/spin_$k.err || exit 2
  TBGPU_BLOCKING_SMALL=1 timeout -k 10 300 $B > $O/block_$k.json 2> $O/block_$k.err || exit 3
done
REPS=2 timeout -k 10 400 python3 profiles/variants.py base noflush skiphot -- --steps 3 --warmup 1 --no-cpu \
  --no-queries --no-subconfigs --no-host > $O/var_c2.txt 2>&1 || exit 4
TB_DIST_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --batches-per-step 100 \
  --accounts 1000000 > $O/bench_routed_gloo2.json 2> $O/bench_routed_gloo2.err || exit 5
