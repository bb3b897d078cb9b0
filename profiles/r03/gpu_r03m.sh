#!/bin/bash
# Round 3: the whole -m gpu suite in one process, with dirty tracking (default) and
# without (TBGPU_NO_INCR=1): do the intermittent general-path mismatches follow it?
OUT=gpurun_out/r03m
mkdir -p "$OUT"
rm -f gpurun_out/tbgpu_fatal.log
for v in default noincr; do
  if [ $v = noincr ]; then E="TBGPU_NO_INCR=1"; else E="TBGPU_UNUSED=1"; fi
  timeout -k 10 600 env $E python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/$v.txt" 2>&1
  rc=$?
  echo "$v rc=$rc: $(tail -1 $OUT/$v.txt)"
  grep "^FAILED" "$OUT/$v.txt"
  cat gpurun_out/tbgpu_fatal.log 2>/dev/null
  { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
done
