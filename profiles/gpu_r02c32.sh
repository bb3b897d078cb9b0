#!/bin/bash
# config 3 A/B on one box: this commit vs the library before fp_tail / k_report
# (build/prev, loaded through TBGPU_LIB), alternating
set -o pipefail
O=gpurun_out/r02c32; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py --config 3 --no-cpu --no-queries --no-host > $O/new_$r.json 2>&1 || exit 1
  TBGPU_LIB=build/prev/libtbgpu.so timeout -k 10 200 python3 -u bench.py --config 3 --no-cpu --no-queries --no-host > $O/prev_$r.json 2>&1 || exit 1
done
for f in $O/*.json; do python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', round(d['value']/1e6,1), d['ms_per_step'], d['roofline'].get('phase_ms_per_step'))"; done
