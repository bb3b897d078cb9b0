# Post/void static records (tr_pv_rec): the general-path GPU tests, then config 3 with and
# without them (TBGPU_NO_PVREC=1), alternating.  OUT=gpurun_out/<dir>.
set -e
OUT=${1:-gpurun_out/pvrec}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_general.py tests/test_gpu_golden.py tests/test_gpu_fuzz.py \
    > $OUT/tests.txt 2>&1
A="--config 3 --steps 5 --warmup 1 --no-cpu --no-queries --no-host"
for r in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export TBGPU_NO_PVREC=1; else unset TBGPU_NO_PVREC; fi
    timeout -k 10 200 python bench.py $A > $OUT/c3_${v}_$r.json 2> $OUT/c3_${v}_$r.err
    echo "$v $r $(python -c "import json;d=json.load(open('$OUT/c3_${v}_$r.json'));print(d['value'],d['ms_per_step'],d['roofline'].get('phase_ms_per_step'))")"
  done
done
