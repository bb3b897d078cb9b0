#!/bin/bash
# r02 rocprofv3 profiles of every bench workload (kernel trace + PMC passes).
set -o pipefail
O=gpurun_out/r02m; mkdir -p $O
export TMPDIR=/tmp
TB_CONFIG=3 TB_ACCOUNTS=10000 TB_CALLS=3 EVENTS_PER_LAUNCH=491400 bash profiles/collect.sh $O/c3 --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host && python3 profiles/summarize.py $O/c3 491400 > $O/c3/summary.txt && echo c3 ok &&
TB_CONFIG=2 TB_ACCOUNTS=1000000 TB_CALLS=3 bash profiles/collect.sh $O/c2 --config 2 --steps 2 --warmup 1 --no-cpu --no-queries --no-host && python3 profiles/summarize.py $O/c2 8190000 > $O/c2/summary.txt && echo c2 ok &&
TB_CONFIG=5 TB_ACCOUNTS=100000000 TB_CALLS=3 bash profiles/collect.sh $O/c5 --config 5 --steps 2 --warmup 1 --no-cpu --no-queries --no-host && python3 profiles/summarize.py $O/c5 8190000 > $O/c5/summary.txt && echo c5 ok &&
TB_CONFIG=4 TB_ACCOUNTS=10000000 TB_CALLS=3 bash profiles/collect.sh $O/c4 --config 4 --steps 2 --warmup 1 --no-cpu --no-queries --no-host && python3 profiles/summarize.py $O/c4 8190000 > $O/c4/summary.txt && echo c4 ok
