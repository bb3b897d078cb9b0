#!/bin/bash
set -o pipefail
O=gpurun_out/r02s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --routed --steps 3 > $O/routed1.json 2> $O/routed1.err; echo "routed1 rc=$?"; cat $O/routed1.json; tail -3 $O/routed1.err
