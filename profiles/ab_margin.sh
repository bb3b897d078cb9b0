set -o pipefail
for i in 1 2 3; do for m in 0 3 6; do
  TBGPU_PASS_MARGIN=$m timeout -k 10 200 python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host > gpurun_out/abm_${m}_${i}.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/abm_${m}_${i}.json')); print('margin', $m, 'rep', $i, round(d['value']/1e6,1), d.get('fixed_point_passes'))"
done; done
