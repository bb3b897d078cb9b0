#!/bin/bash
# round-4 iteration: general-path parity, config-3 timing + trace, config-4 flush ablation
set -o pipefail
O=gpurun_out/${TAG:-r04s4}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_general.py tests/test_gpu_parity.py tests/test_gpu_prefetch.py tests/test_gpu_fuzz.py \
  tests/test_gpu_golden.py tests/test_gpu_checkpoint.py > $O/tests.txt 2>&1 || exit 1
B="python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host"
for k in 1 2; do timeout -k 10 300 $B > $O/c3_$k.json 2> $O/c3_$k.err || exit 2; done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- \
  python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host > $O/kt.log 2>&1 || exit 3
REPS=2 timeout -k 10 400 python3 profiles/variants.py base noflush noret -- --config 4 --steps 3 --warmup 1 --no-cpu \
  --no-queries --no-subconfigs --no-host > $O/var_c4.txt 2>&1 || exit 4
