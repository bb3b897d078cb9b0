# Timing ablations of fp_commit on config 1 with random ids (and sequential for reference):
# FP_ABLATE bits (csrc/fast.h): 2 balances flush, 4 row stores, 32 account probes, 64 id index.
set -e
mkdir -p gpurun_out/abl
A="--config 1 --steps 3 --warmup 1 --no-cpu --no-queries --no-host"
REPS=2 timeout -k 10 900 python3 profiles/variants.py base ids=FP_ABLATE=64 probe=FP_ABLATE=32 both=FP_ABLATE=96 \
    bal=FP_ABLATE=2 rows=FP_ABLATE=4 -- $A --id-order random > gpurun_out/abl/random.txt 2>&1
REPS=2 timeout -k 10 300 python3 profiles/variants.py base probe both -- $A > gpurun_out/abl/seq.txt 2>&1
