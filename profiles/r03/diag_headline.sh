#!/bin/bash
# Round 3: reproduce the driver's headline conditions (bench.py --gpus 1 --steps 20
# --warmup 5 as the first GPU process on a fresh lease) with SMI clock/power samples
# beside every run.  Usage (on the GPU box): bash profiles/r03/diag_headline.sh OUT
OUT=${1:-gpurun_out/r03_diag}
mkdir -p "$OUT"
( while true; do
    echo "=== $(date +%s.%N)"
    timeout 10 amd-smi metric --json 2>&1 | head -c 20000
    timeout 10 rocm-smi --showclocks --showpower --showtemp --json 2>&1 | head -c 4000
    sleep 1
  done ) > "$OUT/smi.log" 2>&1 &
SMI=$!
trap 'kill $SMI 2>/dev/null' EXIT
run() {  # name, env, args
  local name=$1; shift
  echo "== $name start $(date +%s.%N)" >> "$OUT/smi.log"
  timeout -k 10 300 env "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name end rc=$rc $(date +%s.%N)" >> "$OUT/smi.log"
  echo "$name rc=$rc"; tail -c 1500 "$OUT/$name.json" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['frac'], r.get('dominant_ms_per_step'))" || true
  return $rc
}
run first TB_X=1 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-queries --no-host &&
run second TB_X=1 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-queries --no-host &&
run prewarm3 TB_BENCH_PREWARM_S=3 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-queries --no-host &&
run long TB_X=1 python3 bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu --no-queries --no-host &&
run third TB_X=1 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-queries --no-host
