#!/bin/bash
# Round 3: which earlier GPU test file makes a zeroed ctx's create_accounts read zero
# ids (TBGPU_ZERO_ALLOC=1): each file, then the relay-chain test, in one process.
OUT=gpurun_out/r03k
mkdir -p "$OUT"
for f in checkpoint config4 config5 fullsize fuzz; do
  timeout -k 10 400 env TBGPU_ZERO_ALLOC=1 python3 -u -m pytest -q --timeout 200 --timeout-method thread \
    tests/test_gpu_$f.py "tests/test_gpu_general.py::test_adversarial_relay_chain" > "$OUT/$f.txt" 2>&1
  rc=$?
  echo "$f rc=$rc: $(tail -1 $OUT/$f.txt)"
  grep -m3 "^FAILED" "$OUT/$f.txt"
  { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
done
