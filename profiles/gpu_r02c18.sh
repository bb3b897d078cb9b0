#!/bin/bash
# routed step with 2-8 ranks on one GPU (thread-backed collectives): packed wire format at 8 ranks
set -o pipefail
O=gpurun_out/r02c18; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_routed_threads.py -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|passed|failed" $O/tests.txt | tail -14
