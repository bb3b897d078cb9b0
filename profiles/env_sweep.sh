# Config 3 under environment settings of the general path (A/B timing switches), alternating:
#   bash profiles/env_sweep.sh OUT "NAME=VAR=VAL" ...   (NAME=base: no variable)
set -e
OUT=$1; shift
mkdir -p $OUT
A="--config 3 --steps 5 --warmup 1 --no-cpu --no-queries --no-host"
for r in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; kv=${spec#*=}
    if [ "$name" = base ]; then envs=""; else envs="$kv"; fi
    env $envs timeout -k 10 200 python bench.py $A > $OUT/${name}_$r.json 2> $OUT/${name}_$r.err
    echo "$name $r $(python -c "import json;d=json.load(open('$OUT/${name}_$r.json'));print(d['value'],d['ms_per_step'])")"
  done
done
