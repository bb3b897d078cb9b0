#!/bin/bash
# round-4 measurements: the default bench line, then rocprof summaries for config 2 and 3
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
bash profiles/collect.sh $O/c2 > $O/c2.log 2>&1 || exit 2
TB_CONFIG=3 TB_ACCOUNTS=10000 TB_CALLS=3 EVENTS_PER_LAUNCH=491400 \
  bash profiles/collect.sh $O/c3 --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host > $O/c3.log 2>&1 || exit 3
