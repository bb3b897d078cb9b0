#!/bin/bash
# config 3: sparse passes (due stamps checked before the event's loads) against the dense form
set -o pipefail
O=gpurun_out/${TAG:-r04sp}; mkdir -p $O
for r in 1 2; do
  for v in 0 5 4; do
    TBGPU_SPARSE_SHIFT=$v timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu > $O/c3_s$v.$r.json 2> $O/c3_s$v.$r.err || exit 1
  done
done
grep -h -o '"value": [0-9.e+]*' $O/c3_s*.json > $O/summary.txt || true
