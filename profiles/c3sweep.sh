set -e
mkdir -p gpurun_out/c3s
export TBGPU_TRACE_PASSES=1
timeout -k 10 120 python bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-queries --no-host > gpurun_out/c3s/trace.json 2> gpurun_out/c3s/trace.err
unset TBGPU_TRACE_PASSES
for cb in 32 24 40 60; do
  TBGPU_CHUNK_BATCHES=$cb timeout -k 10 150 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu --no-queries --no-host > gpurun_out/c3s/cb$cb.json 2> gpurun_out/c3s/cb$cb.err
  echo "cb $cb $(python -c "import json;d=json.load(open('gpurun_out/c3s/cb$cb.json'));print(d['value'],d['ms_per_step'],d.get('fixed_point_passes'))")"
done
