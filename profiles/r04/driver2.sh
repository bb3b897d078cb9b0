#!/bin/bash
# the driver's command twice on one box (box-to-box spread check)
set -o pipefail
O=gpurun_out/${TAG:-r04d2}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.$r.json 2> $O/bench.$r.err || exit 1
done
