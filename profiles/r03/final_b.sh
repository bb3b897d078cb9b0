#!/bin/bash
# Round 3 evidence on the final code, part B: kernel traces and PMC passes of configs
# 2, 3 and 4 (profiles/collect.sh), the drop-in single-call probe.
#   bash profiles/r03/final_b.sh gpurun_out/r03_final
OUT=${1:-gpurun_out/r03_final}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -20 "$OUT/$name.err"; tail -30 "$OUT/$name.out"; exit $rc; }
}
step pmc_config2 900 env TB_CONFIG=2 TB_ACCOUNTS=1000000 TB_CALLS=3 EVENTS_PER_LAUNCH=8190000 bash profiles/collect.sh "$OUT/pmc_c2" --steps 2 --warmup 1 --no-cpu --no-queries --no-host
grep -A12 "kernel stats" "$OUT/pmc_config2.out" | head -14; grep "fp_commit" "$OUT/pmc_config2.out"
step pmc_config3 900 env TB_CONFIG=3 TB_ACCOUNTS=10000 TB_CALLS=3 EVENTS_PER_LAUNCH=491400 bash profiles/collect.sh "$OUT/pmc_c3" --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host
grep -A12 "kernel stats" "$OUT/pmc_config3.out" | head -14
step pmc_config4 900 env TB_CONFIG=4 TB_ACCOUNTS=10000000 TB_CALLS=3 EVENTS_PER_LAUNCH=8190000 bash profiles/collect.sh "$OUT/pmc_c4" --config 4 --steps 2 --warmup 1 --no-cpu --no-queries --no-host
grep "fp_commit" "$OUT/pmc_config4.out"
step single_call 300 python3 profiles/single_call.py
tail -5 "$OUT/single_call.out"
echo "== done $(date +%T)"
