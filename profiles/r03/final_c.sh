#!/bin/bash
# Round 3, after the create_accounts timestamp fold: the evidence of final_a.sh part 1,
# then a kernel trace of config 4 (its 10M-account create_accounts: ac_mask, ac_ts_fold).
OUT=${1:-gpurun_out/r03_final}
bash profiles/r03/final_a.sh "$OUT" 1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== ac_trace $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ac4" -o ac4 -- \
  python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu --no-queries --no-host > "$OUT/ac4.out" 2> "$OUT/ac4.err" || { echo "ac_trace failed"; tail -5 "$OUT/ac4.err"; exit 1; }
f=$(find "$OUT/ac4" -name "*kernel_stats.csv" | head -1); grep -i "ac_mask\|ac_ts_fold\|ac_apply\|ac_classify" "$f" | cut -c1-200
echo "== done $(date +%T)"
