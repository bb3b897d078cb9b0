#!/bin/bash
# randomized call mixes over the sorted run + hash index
set -o pipefail
O=gpurun_out/r02c19; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "sorted_run" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/tests.txt | head -20
