#!/bin/bash
# Round 3: dirty-tracked passes + the walk's plain cfail store -- whole -m gpu suite,
# then config 3 with and without dirty tracking (TBGPU_NO_INCR), and its kernel trace.
OUT=gpurun_out/r03g
mkdir -p "$OUT"
rm -f gpurun_out/tbgpu_fatal.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.txt"; cat gpurun_out/tbgpu_fatal.log 2>/dev/null
[ $rc -eq 0 ] || exit $rc
for v in incr noincr incr2 noincr2; do
  E=""; case $v in noincr*) E="TBGPU_NO_INCR=1";; esac
  timeout -k 10 300 env $E TB_X=1 python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-queries --no-host > "$OUT/c3_$v.json" 2> "$OUT/c3_$v.err" || exit $?
  python3 profiles/r03/line.py "$OUT/c3_$v.json"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c3 --output-format csv -- python3 bench.py --config 3 --steps 1 --warmup 1 --no-cpu --no-queries --no-host > "$OUT/c3_prof.json" 2> "$OUT/c3_prof.err" || exit $?
find "$OUT/prof" -name "*stats.csv"
