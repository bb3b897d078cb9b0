set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
for B in 60 16 4 1; do
  timeout -k 10 200 python3 bench.py --config 3 --batches-per-step $B --steps 3 --warmup 1 --no-cpu > gpurun_out/b3_$B.json 2> gpurun_out/b3_$B.err || break
  python3 -c "
import json; d=json.load(open('gpurun_out/b3_$B.json')); print($B, round(d['value']/1e6,2), 'M/s', d['ms_per_step'], d['fixed_point_passes'], d['roofline']['phase_ms_per_step'])"
done
