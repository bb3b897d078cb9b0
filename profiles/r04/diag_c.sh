# Round 4 diagnosis: the new create_accounts / prefetch tests, kernel vs copy-engine uploads.
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT; export TMPDIR=/tmp; export TBGPU_FATAL_LOG=$PWD/$OUT/fatal.log
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 200 $PT tests/test_gpu_parity.py -k clean_and_dirty > $OUT/acc_kernel.txt 2>&1; echo "acc_kernel rc=$?"
timeout -k 10 200 env TBGPU_SDMA_H2D=1 $PT tests/test_gpu_parity.py -k clean_and_dirty > $OUT/acc_sdma.txt 2>&1; echo "acc_sdma rc=$?"
timeout -k 10 200 env TBGPU_NO_AC_FAST=1 $PT tests/test_gpu_parity.py -k clean_and_dirty > $OUT/acc_nofast.txt 2>&1; echo "acc_nofast rc=$?"
timeout -k 10 200 env TBGPU_SDMA_H2D=1 $PT tests/test_gpu_prefetch.py > $OUT/pf_sdma.txt 2>&1; echo "pf_sdma rc=$?"
timeout -k 10 200 $PT tests/test_gpu_prefetch.py > $OUT/pf_kernel.txt 2>&1; echo "pf_kernel rc=$?"
