#!/bin/bash
set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config 3 --no-queries --no-host --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err; echo "c3 rc=$?"; cat $O/bench_c3.json
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt3 -o kt --output-format csv -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/kt3.log 2>&1; echo "kt3 rc=$?"
python3 profiles/summarize.py $O > $O/kt3_summary.txt 2>&1; cat $O/kt3_summary.txt | head -30
