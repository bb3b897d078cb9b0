#!/bin/bash
# r02 evidence after the router changes: GPU tests, smoke, the driver's bench command,
# every config (1-5, routed), kernel traces of configs 1 and 2
set -o pipefail
O=gpurun_out/r02c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.txt
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; echo "bench rc=$? $(grep -o '"value": [0-9.]*' $O/bench.json | head -1) $(grep -o '"frac": [0-9.]*' $O/bench.json | head -1)"
timeout -k 10 300 python3 -u bench.py --config 1 --no-queries > $O/bench_config1.json 2> $O/bench_config1.err; echo "c1 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config1.json | head -1)"
timeout -k 10 300 python3 -u bench.py --config 3 --no-queries --verify > $O/bench_config3.json 2> $O/bench_config3.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config3.json | head -1)"
timeout -k 10 300 python3 -u bench.py --config 4 --no-queries > $O/bench_config4.json 2> $O/bench_config4.err; echo "c4 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config4.json | head -1)"
timeout -k 10 600 python3 -u bench.py --config 5 --no-queries > $O/bench_config5.json 2> $O/bench_config5.err; echo "c5 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config5.json | head -1)"
timeout -k 10 400 python3 -u bench.py --routed --steps 4 --no-cpu > $O/bench_routed_1rank.json 2> $O/bench_routed_1rank.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/bench_routed_1rank.json)"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/kt_c2.log 2>&1; echo "kt c2 rc=$?"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt_c1 -o kt --output-format csv -- python3 bench.py --config 1 --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/kt_c1.log 2>&1; echo "kt c1 rc=$?"
