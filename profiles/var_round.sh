# Parity of each timing variant on the fast-path tests, then variants.py timing.
#   bash profiles/var_round.sh NAME...   (GPU box, repo root; build/var_NAME built beforehand)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  [ "$v" = -- ] && break
  [ "$v" = base ] && continue
  TBGPU_LIB=tigerbeetle_amd/build/var_$v/libtbgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
    --timeout 120 --timeout-method thread -k "config1 or config2 or fast or random or config4" > gpurun_out/par_$v.log 2>&1 \
    || { echo "parity FAILED for $v"; tail -20 gpurun_out/par_$v.log; exit 1; }
  echo "parity ok: $v $(tail -1 gpurun_out/par_$v.log)"
done
REPS=${REPS:-3} timeout -k 10 600 python -u profiles/variants.py "$@" | tee gpurun_out/variants.txt
