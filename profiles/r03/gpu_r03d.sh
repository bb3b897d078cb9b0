#!/bin/bash
# Round 3: fp_commit variants on config 2 -- coalesced row stores through the wave's
# stage (FP_STAGE_ROWS), and the timing-only no-flush / no-return flush -- parity of the
# kept candidate first, then alternating fresh processes on one box (cached workload).
OUT=gpurun_out/r03d
mkdir -p "$OUT"
V=tigerbeetle_amd/build
timeout -k 10 600 env TBGPU_LIB=$V/var_stagerows/libtbgpu.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > "$OUT/parity_stagerows.txt" 2>&1 || { tail -30 "$OUT/parity_stagerows.txt"; exit 1; }
tail -1 "$OUT/parity_stagerows.txt"
export TB_BENCH_CACHE=/tmp/tbcache
ARGS="--steps 5 --warmup 2 --no-cpu --no-queries --no-host"
REPS=1 timeout -k 10 900 python3 profiles/variants.py base stagerows noflush noret base stagerows base stagerows -- $ARGS > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
# the fuzz case that aborted in r03c (last: an abort ends the call)
timeout -k 10 300 python -u -m pytest "tests/test_gpu_fuzz.py::test_fuzz_mutations[19]" -x -q -s --timeout 120 --timeout-method thread > "$OUT/fuzz19.txt" 2>&1
echo "fuzz19 rc=$?"; grep -v "^  File\|^    " "$OUT/fuzz19.txt" | head -40
