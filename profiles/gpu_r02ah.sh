#!/bin/bash
# fp_commit flush ablation on config 4 and config 2 (timing only: noflush results are wrong)
set -o pipefail
export TMPDIR=/tmp
REPS=2 timeout -k 10 500 python -u profiles/variants.py base noflush noret -- --config 4 --steps 3 --warmup 1 --no-cpu --no-queries --no-host
REPS=2 timeout -k 10 400 python -u profiles/variants.py base noflush noret -- --steps 3 --warmup 1 --no-cpu --no-queries --no-host
