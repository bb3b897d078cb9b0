#!/bin/bash
# Round 2, first GPU call: the new general-path tests, then the config-3 bench (retuned
# to ~10 % non-ok) and its kernel trace, the default bench, and the counter list.
set -o pipefail
mkdir -p gpurun_out/r02a
O=gpurun_out/r02a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_general.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/gpu_tests_general.log 2>&1; echo "tests rc=$?"; tail -5 $O/gpu_tests_general.log
timeout -k 10 300 python -u bench.py --config 3 --no-queries > $O/bench_c3.json 2> $O/bench_c3.err; echo "c3 rc=$?"; cat $O/bench_c3.json
timeout -k 10 300 python -u bench.py --no-queries > $O/bench_c2.json 2> $O/bench_c2.err; echo "c2 rc=$?"; cat $O/bench_c2.json
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt3 -o kt -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/kt3.log 2>&1; echo "kt3 rc=$?"
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "L rc=$?"
python3 profiles/summarize.py $O/kt3 > $O/kt3_summary.txt 2>&1; head -30 $O/kt3_summary.txt
