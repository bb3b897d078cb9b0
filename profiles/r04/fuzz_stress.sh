#!/bin/bash
# the wider randomized sweep (tests/test_gpu_fuzz.py test_fuzz_stress_sweep): 20000 small
# seeds, then 300 with full-size batches; each whole-call and on the forced general path
# (every 5th also batch by batch, every 7th walked after two passes), every reply and the
# whole state vs the oracle
set -o pipefail
O=gpurun_out/${TAG:-r04fz}; mkdir -p $O
TB_FUZZ_STRESS=96:20000 timeout -k 10 900 python3 -u -m pytest -x -q -s --timeout 880 --timeout-method thread \
  tests/test_gpu_fuzz.py -k stress > $O/fuzz_small.txt 2>&1 || exit 1
TB_FUZZ_BIG=1 TB_FUZZ_STRESS=50000:300 timeout -k 10 600 python3 -u -m pytest -x -q -s --timeout 580 --timeout-method thread \
  tests/test_gpu_fuzz.py -k stress > $O/fuzz_big.txt 2>&1 || exit 2
