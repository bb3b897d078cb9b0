#!/bin/bash
# round-4 iteration: the whole GPU suite, then the driver's command (host_path: fp_tail's report)
set -o pipefail
O=gpurun_out/${TAG:-r04s5}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 2
TBGPU_NO_TAIL_REPORT=1 timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --no-queries \
  --no-subconfigs > $O/bench_notailreport.json 2> $O/bench_ntr.err || exit 3
