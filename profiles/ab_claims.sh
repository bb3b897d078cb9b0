# Store-claims + fp_claim_verify (round 5): the eager-claim tests and the random-id fuzz,
# then config 1 with random ids.  OUT=gpurun_out/<dir>.
set -e
OUT=${1:-gpurun_out/claims}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py tests/test_gpu_prefetch.py \
    > $OUT/tests.txt 2>&1
for r in 1 2; do
  timeout -k 10 200 python bench.py --config 1 --id-order random --steps 5 --warmup 1 --no-cpu --no-queries --no-host \
      > $OUT/c1r_$r.json 2> $OUT/c1r_$r.err
  echo "random $r $(python -c "import json;d=json.load(open('$OUT/c1r_$r.json'));print(d['value'],d['ms_per_step'],d['roofline']['phase_ms_per_step'])")"
done
