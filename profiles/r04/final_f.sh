#!/bin/bash
# round-4 closing set on the last engine commit: smoke, the driver's command, config 3's line,
# its kernel trace and PMC passes
set -o pipefail
O=gpurun_out/${TAG:-r04ff}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 300 python3 -u bench.py --config 3 > $O/bench_config3.json 2> $O/bench_config3.err || exit 3
TB_CONFIG=3 TB_ACCOUNTS=10000 TB_CALLS=3 EVENTS_PER_LAUNCH=491400 \
  bash profiles/collect.sh $O/c3 --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host > $O/c3.log 2>&1 || exit 4
