#!/bin/bash
# drop-in single call: blocking vs polling waits (TBGPU_POLL_SYNC=1), alternating on one box
set -o pipefail
O=gpurun_out/r02c34; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 -u profiles/single_call.py 512 > $O/block_$r.txt 2>&1 || exit 1; tail -1 $O/block_$r.txt
  TBGPU_POLL_SYNC=1 timeout -k 10 200 python3 -u profiles/single_call.py 512 > $O/poll_$r.txt 2>&1 || exit 1; tail -1 $O/poll_$r.txt
done
