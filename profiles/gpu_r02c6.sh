#!/bin/bash
# sorted-run id index: full GPU suite, config 2 (driver command) and config 4/5 lines
set -o pipefail
O=gpurun_out/r02c6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-queries > $O/bench.json 2> $O/bench.err; echo "bench rc=$? $(grep -o '"value": [0-9.]*' $O/bench.json | head -1) $(grep -o '"frac": [0-9.]*' $O/bench.json | head -1)"
timeout -k 10 300 python3 -u bench.py --config 4 --no-queries --no-cpu > $O/bench_config4.json 2> $O/bench_config4.err; echo "c4 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config4.json | head -1)"
timeout -k 10 400 python3 -u bench.py --routed --steps 6 --no-cpu > $O/routed.json 2> $O/routed.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/routed.json)"
