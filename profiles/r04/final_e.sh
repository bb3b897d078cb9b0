#!/bin/bash
# round-4 closing set on the last engine commit: the GPU suite, smoke, the driver's command, config 3
set -o pipefail
O=gpurun_out/${TAG:-r04fe}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 3
timeout -k 10 300 python3 -u bench.py --config 3 > $O/bench_config3.json 2> $O/bench_config3.err || exit 4
