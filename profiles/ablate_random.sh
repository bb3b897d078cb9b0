# Timing ablations of fp_commit on config 1 with random ids:
# FP_ABLATE bits (csrc/fast.h): 64 id index, 256 the claim as a plain store at the probe's end
# slot for every event, 512 the product's store-claim also where classify read no slot.
set -e
mkdir -p gpurun_out/abl
A="--config 1 --steps 3 --warmup 1 --no-cpu --no-queries --no-host"
REPS=2 timeout -k 10 900 python3 profiles/variants.py base cstore=FP_ABLATE=256 storeall=FP_ABLATE=512 \
    -- $A --id-order random > gpurun_out/abl/random4.txt 2>&1
