#!/bin/bash
# general path: apply kernels enqueued behind every pass group, gated on a device convergence word
set -o pipefail
O=gpurun_out/r02c20; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u bench.py --config 3 --no-queries --no-cpu --no-host --verify > $O/c3v.json 2> $O/c3v.err; echo "c3 verify rc=$? $(grep -o '"value": [0-9.]*' $O/c3v.json | head -1) $(grep -o '"replies_bit_exact": [a-z]*' $O/c3v.json) $(grep -o '"accounts_bit_exact": [a-z]*' $O/c3v.json)"
for r in 1 2; do timeout -k 10 300 python3 -u bench.py --config 3 --steps 4 --no-queries --no-cpu --no-host > $O/c3_$r.json 2> $O/c3_$r.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/c3_$r.json | head -1)"; done
