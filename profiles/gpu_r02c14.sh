#!/bin/bash
# batch block copy fixed (the chunk's starts + timestamps only): configs 2 (+ host path), 3, routed
set -o pipefail
O=gpurun_out/r02c14; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_general.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --no-queries --no-cpu > $O/c2.json 2> $O/c2.err; echo "c2 rc=$? $(grep -o '"value": [0-9.]*' $O/c2.json | head -1) $(grep -o '"upload": [0-9.]*' $O/c2.json) $(grep -o '"single": {[^}]*}' $O/c2.json)"
for r in 1 2; do timeout -k 10 300 python3 -u bench.py --config 3 --steps 4 --no-queries --no-cpu --no-host > $O/c3_$r.json 2> $O/c3_$r.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/c3_$r.json | head -1)"; done
timeout -k 10 300 python3 -u bench.py --routed --steps 6 --no-cpu > $O/routed.json 2> $O/routed.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/routed.json | head -1)"
