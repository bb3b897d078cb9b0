#!/bin/bash
# config-2 fp_commit ablation (timing variants, results wrong by design): the flush, the hot rows
set -o pipefail
O=gpurun_out/${TAG:-r04v}; mkdir -p $O
[ -n "$SKIP_PERM" ] || REPS=2 timeout -k 10 500 python3 profiles/variants.py base noflush skiphot base -- --steps 3 --warmup 1 --no-cpu \
  --no-queries --no-subconfigs --no-host > $O/var_c2.txt 2>&1 || exit 1
# the same with rank r at row r (TB_ZIPF_IDENTITY=1), so that FP_SKIP_HOT=1024 drops the 1024 hottest accounts' atomics
TB_ZIPF_IDENTITY=1 REPS=2 timeout -k 10 500 python3 profiles/variants.py base skiphot base -- --steps 3 --warmup 1 --no-cpu \
  --no-queries --no-subconfigs --no-host > $O/var_c2_identity.txt 2>&1 || exit 2
