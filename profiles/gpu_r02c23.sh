#!/bin/bash
# routed one-rank: kernel traces of the plain and the pipelined stream
set -o pipefail
O=gpurun_out/r02c23; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_plain -o kt --output-format csv -- python3 bench.py --routed --steps 6 --no-cpu > $O/plain.json 2> $O/plain.log; echo "plain rc=$?"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_pipe -o kt --output-format csv -- python3 bench.py --routed --pipelined --steps 6 --no-cpu > $O/pipe.json 2> $O/pipe.log; echo "pipe rc=$?"
