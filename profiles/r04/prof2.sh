#!/bin/bash
# round-4 rocprof summaries: config 2 (the driver's workload) and config 4, kernel trace + PMC
set -o pipefail
O=gpurun_out/r04p2; mkdir -p $O
bash profiles/collect.sh $O/c2 > $O/c2.log 2>&1 || exit 1
TB_CONFIG=4 TB_ACCOUNTS=10000000 bash profiles/collect.sh $O/c4 --config 4 --steps 2 --warmup 1 --no-cpu --no-queries \
  --no-subconfigs --no-host > $O/c4.log 2>&1 || exit 2
TBGPU_EVAL_PROBE=1 timeout -k 10 200 python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-queries \
  --no-subconfigs --no-host > $O/probe.json 2> $O/probe.err || exit 3
