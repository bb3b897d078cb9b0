#!/bin/bash
# fp_commit without the id key copies (sorted run) vs with them; parity first
set -o pipefail
O=gpurun_out/r02c11; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py tests/test_gpu_checkpoint.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit 1
REPS=3 timeout -k 10 500 python -u profiles/variants.py base keys -- --steps 8 --warmup 2 --no-cpu --no-queries --no-host > $O/var_c2.txt 2>&1; echo "c2 rc=$?"; cat $O/var_c2.txt
