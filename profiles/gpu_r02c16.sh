#!/bin/bash
# config 2 across fresh processes on one box, with and without an untimed HBM pre-warm
set -o pipefail
O=gpurun_out/r02c16; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for pw in 0 400; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --no-queries --no-host --prewarm-ms $pw > $O/c2_${pw}_$r.json 2> $O/c2_${pw}_$r.err
    echo "prewarm=$pw run=$r rc=$? $(grep -o '"value": [0-9.]*' $O/c2_${pw}_$r.json | head -1) $(grep -o '"classify": [0-9.]*' $O/c2_${pw}_$r.json)"
  done
done
