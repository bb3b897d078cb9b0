#!/bin/bash
# Round 3: test_queries_flag_mix_with_history fails after the parity file in one process.
OUT=gpurun_out/r03o
mkdir -p "$OUT"
run() {  # name, env, pytest args...
  local name=$1 e=$2; shift 2
  timeout -k 10 300 env $e python3 -u -m pytest -q --timeout 200 --timeout-method thread "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $OUT/$name.txt)"; grep "^FAILED" "$OUT/$name.txt"
  { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
}
Q=tests/test_gpu_queries.py
run queries_alone TBGPU_UNUSED=1 $Q
run queries_alone_zero TBGPU_ZERO_ALLOC=1 $Q
run parity_then_queries TBGPU_UNUSED=1 tests/test_gpu_parity.py $Q
run fullsize_then_queries TBGPU_UNUSED=1 tests/test_gpu_fullsize.py $Q
