#!/bin/bash
# Config 3 under the engine's tuning switches (env), alternating in fresh processes:
#   bash profiles/env_sweep.sh OUT REPS "VAR=a" "VAR=b" ...   (an empty spec is the default)
set -o pipefail
OUT=${1:?}; REPS=${2:?}; shift 2
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for spec in "$@"; do
    tag=${spec:-default}; tag=${tag//\//_}
    env $spec timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu --no-queries --no-host \
      --no-subconfigs > "$OUT/$tag.$rep.json" 2> "$OUT/$tag.$rep.err" || exit 1
    python3 -c "
import json; d=json.loads(open('$OUT/$tag.$rep.json').read().strip().splitlines()[-1])
print('$tag', $rep, round(d['value']/1e6,1), d['ms_per_step'], d.get('fixed_point_passes'), flush=True)"
  done
done
