#!/bin/bash
# polled vs blocking stream waits (TBGPU_BLOCKING_SYNC=1): configs 3, 2 (+ host path), routed
set -o pipefail
O=gpurun_out/r02c13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_general.py tests/test_gpu_parity.py tests/test_gpu_routed_threads.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit 1
for m in poll block; do
  if [ $m = block ]; then export TBGPU_BLOCKING_SYNC=1; fi
  timeout -k 10 300 python3 -u bench.py --config 3 --steps 4 --no-queries --no-cpu --no-host > $O/c3_$m.json 2> $O/c3_$m.err; echo "$m c3 rc=$? $(grep -o '"value": [0-9.]*' $O/c3_$m.json | head -1)"
  timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --no-queries --no-cpu > $O/c2_$m.json 2> $O/c2_$m.err; echo "$m c2 rc=$? $(grep -o '"value": [0-9.]*' $O/c2_$m.json | head -1) $(grep -o '"single": {[^}]*}' $O/c2_$m.json)"
  timeout -k 10 300 python3 -u bench.py --routed --steps 6 --no-cpu > $O/routed_$m.json 2> $O/routed_$m.err; echo "$m routed rc=$? $(grep -o '"value": [0-9.]*' $O/routed_$m.json | head -1)"
done
