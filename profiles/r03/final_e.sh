#!/bin/bash
# Round 3, final engine: the driver's bench command, then a kernel trace of config 4
# (its 10M-account create_accounts: ac_mask and ac_ts_fold).
OUT=${1:-gpurun_out/r03_final}
mkdir -p "$OUT"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.out" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python3 profiles/r03/line.py "$OUT/bench.out"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ac4" -o ac4 -- \
  python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu --no-queries --no-host > "$OUT/ac4.out" 2> "$OUT/ac4.err" || { echo "trace failed"; tail -5 "$OUT/ac4.err"; exit 1; }
f=$(find "$OUT/ac4" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_config4_accounts.csv"; grep -i "ac_mask\|ac_ts_fold\|ac_apply\|ac_classify\|fp_commit" "$f" | cut -c1-160
