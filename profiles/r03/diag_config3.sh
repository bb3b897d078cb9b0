#!/bin/bash
# Round 3: config 3 (general path) chunk-size sweep with pass traces, then a kernel
# trace of the default.  Usage (GPU box): bash profiles/r03/diag_config3.sh OUT
OUT=${1:-gpurun_out/r03_c3}
mkdir -p "$OUT"
ARGS="python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host"
for cb in 20 40 60; do
  timeout -k 10 300 env TBGPU_CHUNK_BATCHES=$cb TBGPU_TRACE_PASSES=1 $ARGS > "$OUT/c3_cb$cb.json" 2> "$OUT/c3_cb$cb.err" || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/c3_cb$cb.json').read().strip().splitlines()[-1]); print('cb=$cb', round(d['value']/1e6,1), 'M/s', d['roofline']['phase_ms_per_step'])"
  grep -c "pass" "$OUT/c3_cb$cb.err"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c3 -- python3 bench.py --config 3 --steps 1 --warmup 1 --no-cpu --no-queries --no-host > "$OUT/c3_prof.json" 2> "$OUT/c3_prof.err"
