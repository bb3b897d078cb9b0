#!/bin/bash
# the driver's command, then each BASELINE config's line
set -o pipefail
O=gpurun_out/${TAG:-r04b}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
for c in 1 3 4 5; do
  timeout -k 10 400 python3 -u bench.py --config $c > $O/bench_config$c.json 2> $O/bench_config$c.err || exit 2
done
timeout -k 10 400 python3 -u bench.py --config 4 --routed > $O/bench_routed_1rank.json 2> $O/bench_routed.err || exit 3
