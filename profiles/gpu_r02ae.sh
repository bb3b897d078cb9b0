#!/bin/bash
# re-entry baseline: config 3 with per-pass change counts, routed one-rank phases
set -o pipefail
O=gpurun_out/r02ae; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --config 3 --no-queries --no-host --cpu-seconds 2 > $O/c3.json 2> $O/c3.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/c3.json | head -1)"
TBGPU_TRACE_PASSES=1 timeout -k 10 300 python3 -u bench.py --config 3 --no-queries --no-host --no-cpu --steps 1 --warmup 0 > $O/c3trace.json 2> $O/c3trace.err; echo "c3trace rc=$?"
timeout -k 10 400 python3 -u bench.py --routed --steps 4 --no-cpu > $O/routed.json 2> $O/routed.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/routed.json)"
