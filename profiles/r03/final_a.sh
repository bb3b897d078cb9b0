#!/bin/bash
# Round 3 evidence on the final code, part A (one gpurun call, fresh MI355X):
#   bash profiles/r03/final_a.sh gpurun_out/r03_final [1|2]   (part 1, part 2, or both)
# the -m gpu suite, smoke, the driver's bench command, every BASELINE config's line,
# config 3 with and without dirty tracking, the routed one-rank and gloo two-rank lines.
OUT=${1:-gpurun_out/r03_final}
PART=${2:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, seconds, command...: one GPU step under its own limit; stop at the first failure
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -20 "$OUT/$name.err"; tail -30 "$OUT/$name.out"; cat gpurun_out/tbgpu_fatal.log 2>/dev/null; exit $rc; }
}
rm -f gpurun_out/tbgpu_fatal.log
if [ "$PART" != 2 ]; then
# the suite: test failures (rc 1) are reported and the evidence goes on; anything else stops
echo "== gpu_tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.out" 2> "$OUT/gpu_tests.err"
rc=$?
tail -2 "$OUT/gpu_tests.out"; grep "^FAILED\|^E   .*AssertionError" "$OUT/gpu_tests.out" | cut -c1-600
{ [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || { echo "gpu_tests rc=$rc"; cat gpurun_out/tbgpu_fatal.log 2>/dev/null; exit $rc; }
step smoke 180 python3 -u __graft_entry__.py smoke
cat "$OUT/smoke.out"
step bench 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
python3 profiles/r03/line.py "$OUT/bench.out"
step bench_config3 400 python3 bench.py --config 3 --no-queries --no-host
python3 profiles/r03/line.py "$OUT/bench_config3.out"
step bench_config3_noincr 400 env TBGPU_NO_INCR=1 python3 bench.py --config 3 --no-cpu --no-queries --no-host
python3 profiles/r03/line.py "$OUT/bench_config3_noincr.out"
fi
[ "$PART" = 1 ] && { echo "== done $(date +%T)"; exit 0; }
for c in 1 4 5; do
  step bench_config$c 400 python3 bench.py --config $c --no-queries --no-host
  python3 profiles/r03/line.py "$OUT/bench_config$c.out"
done
step bench_routed_1rank 400 python3 bench.py --routed --no-queries
python3 profiles/r03/line.py "$OUT/bench_routed_1rank.out"
step bench_routed_gloo2 600 env TB_DIST_BACKEND=gloo python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --batches-per-step 100 --accounts 1000000
python3 profiles/r03/line.py "$OUT/bench_routed_gloo2.out"
echo "== done $(date +%T)"
