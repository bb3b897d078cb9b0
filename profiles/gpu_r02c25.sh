#!/bin/bash
# speculative fast attempt with grid-stride gated fix launches; A/B with TBGPU_NO_SPEC=1
set -o pipefail
O=gpurun_out/r02c25; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for m in spec nospec; do
    if [ $m = nospec ]; then export TBGPU_NO_SPEC=1; else unset TBGPU_NO_SPEC; fi
    timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-queries --no-cpu > $O/c2_${m}_$r.json 2> $O/c2_${m}_$r.err; echo "$m c2 rc=$? $(grep -o '"value": [0-9.]*' $O/c2_${m}_$r.json | head -1) $(grep -o '"classify": [0-9.]*' $O/c2_${m}_$r.json) $(grep -o '"single": {[^}]*}' $O/c2_${m}_$r.json | grep -o '"p50": [0-9.]*')"
  done
done
