#!/bin/bash
set -o pipefail
O=gpurun_out/r02aa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_routed_threads.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|error" $O/t.log | head -20
