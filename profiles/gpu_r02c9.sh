#!/bin/bash
# fp_chains: 16 results per lane; parity + config 4
set -o pipefail
O=gpurun_out/r02c9; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_routed_threads.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u bench.py --config 4 --steps 6 --no-queries --no-cpu --no-host > $O/c4.json 2> $O/c4.err; echo "c4 rc=$? $(grep -o '"value": [0-9.]*' $O/c4.json | head -1) $(grep -o '"phase_ms_per_step": {[^}]*}' $O/c4.json)"
timeout -k 10 400 python3 -u bench.py --routed --steps 6 --no-cpu > $O/routed.json 2> $O/routed.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/routed.json)"
