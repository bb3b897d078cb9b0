#!/bin/bash
# config 3 (and config 2's host path): blocking vs polled stream waits, alternating
set -o pipefail
O=gpurun_out/r02c22; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for m in block poll; do
    if [ $m = poll ]; then export TBGPU_POLL_SYNC=1; else unset TBGPU_POLL_SYNC; fi
    timeout -k 10 300 python3 -u bench.py --config 3 --steps 4 --no-queries --no-cpu --no-host > $O/c3_${m}_$r.json 2> $O/c3_${m}_$r.err; echo "$m c3 rc=$? $(grep -o '"value": [0-9.]*' $O/c3_${m}_$r.json | head -1)"
  done
done
