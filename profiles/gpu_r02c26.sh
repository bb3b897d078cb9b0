#!/bin/bash
# config 2: does the bench's footprint (25 steps of events and rows resident) move fp_commit?
# alternating the driver command and a 3-step run on one box
set -o pipefail
O=gpurun_out/r02c26; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-queries --no-host > $O/big_$r.json 2> $O/big_$r.err; echo "big run=$r rc=$? $(grep -o '"value": [0-9.]*' $O/big_$r.json | head -1) $(grep -o '"classify": [0-9.]*' $O/big_$r.json)"
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/small_$r.json 2> $O/small_$r.err; echo "small run=$r rc=$? $(grep -o '"value": [0-9.]*' $O/small_$r.json | head -1) $(grep -o '"classify": [0-9.]*' $O/small_$r.json)"
done
