#!/bin/bash
set -o pipefail
O=gpurun_out/r02n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_shard.log 2>&1; rc=$?; echo "shard tests rc=$rc"; tail -2 $O/gpu_shard.log
[ $rc -eq 0 ] || exit 1
TB_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --batches-per-step 100 --steps 2 --accounts 1000000 > $O/routed2.json 2> $O/routed2.err; echo "routed rc=$?"; cat $O/routed2.json; tail -3 $O/routed2.err
