#!/bin/bash
# r02 final evidence, part A: GPU tests, smoke, the driver's bench command, every config
set -o pipefail
O=gpurun_out/r02final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.txt
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; echo "bench rc=$? $(grep -o '"value": [0-9.]*' $O/bench.json) $(grep -o '"frac": [0-9.]*' $O/bench.json | head -1)"
timeout -k 10 300 python3 -u bench.py --config 3 --no-queries > $O/bench_config3.json 2> $O/bench_config3.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config3.json | head -2)"
timeout -k 10 300 python3 -u bench.py --config 4 --no-queries > $O/bench_config4.json 2> $O/bench_config4.err; echo "c4 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config4.json | head -2)"
timeout -k 10 600 python3 -u bench.py --config 5 --no-queries > $O/bench_config5.json 2> $O/bench_config5.err; echo "c5 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config5.json | head -2)"
timeout -k 10 400 python3 -u bench.py --routed --steps 4 --no-cpu > $O/bench_routed_1rank.json 2> $O/bench_routed_1rank.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/bench_routed_1rank.json)"
