#!/bin/bash
# the wider randomized sweep (tests/test_gpu_fuzz.py test_fuzz_stress_sweep): seeds 96..1095,
# each whole-call and on the forced general path, every reply and the state vs the oracle
set -o pipefail
O=gpurun_out/${TAG:-r04fz}; mkdir -p $O
TB_FUZZ_STRESS=96:1000 timeout -k 10 1000 python3 -u -m pytest -x -q -s --timeout 950 --timeout-method thread \
  tests/test_gpu_fuzz.py -k stress > $O/fuzz_stress.txt 2>&1 || exit 1
