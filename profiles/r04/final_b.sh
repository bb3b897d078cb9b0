#!/bin/bash
# round-4 closing set, part B: every config's line, the routed N=1 line, config 3's traces and PMC
set -o pipefail
O=gpurun_out/${TAG:-r04fb}; mkdir -p $O
export TMPDIR=/tmp
for c in 1 3 4 5; do
  timeout -k 10 400 python3 -u bench.py --config $c > $O/bench_config$c.json 2> $O/bench_config$c.err || exit 1
done
timeout -k 10 400 python3 -u bench.py --config 4 --routed > $O/bench_routed_1rank.json 2> $O/bench_routed.err || exit 2
TB_CONFIG=3 TB_ACCOUNTS=10000 TB_CALLS=3 EVENTS_PER_LAUNCH=491400 \
  bash profiles/collect.sh $O/c3 --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host > $O/c3.log 2>&1 || exit 3
