#!/bin/bash
# Round 3: the whole -m gpu suite in one process with every allocation zeroed
# (TBGPU_ZERO_ALLOC=1), then as shipped: do the long-process failures come from reads
# of memory an earlier ctx left behind?
OUT=gpurun_out/r03n
mkdir -p "$OUT"
rm -f gpurun_out/tbgpu_fatal.log
for v in zero default; do
  if [ $v = zero ]; then E="TBGPU_ZERO_ALLOC=1"; else E="TBGPU_UNUSED=1"; fi
  timeout -k 10 600 env $E python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/$v.txt" 2>&1
  rc=$?
  echo "$v rc=$rc: $(tail -1 $OUT/$v.txt)"
  grep "^FAILED" "$OUT/$v.txt"
  cat gpurun_out/tbgpu_fatal.log 2>/dev/null
  { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
done
