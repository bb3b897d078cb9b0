#!/bin/bash
# r02 final evidence, part B: rocprofv3 kernel traces and PMC passes (configs 3 and 2)
set -o pipefail
O=gpurun_out/r02final; mkdir -p $O
export TMPDIR=/tmp
TB_CONFIG=3 TB_ACCOUNTS=10000 TB_CALLS=3 EVENTS_PER_LAUNCH=491400 bash profiles/collect.sh $O/c3 --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host && python3 profiles/summarize.py $O/c3 491400 > $O/c3/summary.txt && echo c3 ok &&
TB_CONFIG=2 TB_ACCOUNTS=1000000 TB_CALLS=3 bash profiles/collect.sh $O/c2 --config 2 --steps 2 --warmup 1 --no-cpu --no-queries --no-host && python3 profiles/summarize.py $O/c2 8190000 > $O/c2/summary.txt && echo c2 ok &&
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_routed -o kt --output-format csv -- python3 bench.py --routed --steps 2 --no-cpu > $O/kt_routed.log 2>&1 && echo routed kt ok
