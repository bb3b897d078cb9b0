#!/bin/bash
# routed one-rank: unpipelined vs pipelined after the packed-format / scatter changes
set -o pipefail
O=gpurun_out/r02c2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --routed --steps 6 --no-cpu > $O/routed.json 2> $O/routed.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/routed.json)"
timeout -k 10 400 python3 -u bench.py --routed --pipelined --steps 6 --no-cpu > $O/routed_pipe.json 2> $O/routed_pipe.err; echo "pipelined rc=$? $(grep -o '"value": [0-9.]*' $O/routed_pipe.json)"
