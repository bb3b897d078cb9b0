#!/bin/bash
# config 2 repeatability on one box (fp_commit time across three fresh processes)
set -o pipefail
O=gpurun_out/r02c15; mkdir -p $O
export TMPDIR=/tmp
REPS=3 timeout -k 10 500 python -u profiles/variants.py base -- --steps 8 --warmup 2 --no-cpu --no-queries --no-host > $O/var_c2.txt 2>&1; echo "c2 rc=$?"; cat $O/var_c2.txt
rocm-smi --showclocks --showpower > $O/smi.txt 2>&1; grep -iE "sclk|mclk|power" $O/smi.txt | head -6
