#!/bin/bash
# kernel traces of config 3: incremental passes vs every pass full
set -o pipefail
O=gpurun_out/r02ag; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --config 3 --steps 1 --warmup 1 --no-cpu --no-queries --no-host"
timeout -s KILL 150 rocprofv3 --kernel-trace -d $O/inc -o kt --output-format csv -- $B > $O/inc.log 2>&1; echo "inc rc=$?"
TBGPU_FULL_PASSES=1 timeout -s KILL 150 rocprofv3 --kernel-trace -d $O/full -o kt --output-format csv -- $B > $O/full.log 2>&1; echo "full rc=$?"
python3 profiles/passtrace.py $O/inc > $O/inc.txt; tail -25 $O/inc.txt
python3 profiles/passtrace.py $O/full > $O/full.txt; tail -25 $O/full.txt
