#!/bin/bash
# config 2: how much of fp_commit's flush is the hottest accounts' same-address atomics
# (timing-only variants: skip the flush of rows < 64 / < 1024; no flush at all)
set -o pipefail
O=gpurun_out/r02c28; mkdir -p $O
export TMPDIR=/tmp
REPS=2 timeout -k 10 600 python -u profiles/variants.py base hot64 hot1k noflush base -- --steps 8 --warmup 2 --no-cpu --no-queries --no-host > $O/var.txt 2>&1; echo "rc=$?"; cat $O/var.txt
