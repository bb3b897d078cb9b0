#!/bin/bash
# fp_commit: 16-record staging (3 workgroups per CU) vs 32 (2 per CU), configs 2 and 4
set -o pipefail
O=gpurun_out/r02c7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.txt
[ $rc -eq 0 ] || exit 1
REPS=3 timeout -k 10 500 python -u profiles/variants.py base s32 -- --steps 8 --warmup 2 --no-cpu --no-queries --no-host > $O/var_c2.txt 2>&1; echo "c2 rc=$?"; cat $O/var_c2.txt
REPS=2 timeout -k 10 500 python -u profiles/variants.py base s32 -- --config 4 --steps 6 --warmup 1 --no-cpu --no-queries --no-host > $O/var_c4.txt 2>&1; echo "c4 rc=$?"; cat $O/var_c4.txt
