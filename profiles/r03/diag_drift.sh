#!/bin/bash
# Round 3: the config-2 drift across processes on one box.  Alternates the product
# library (hot tables physically contiguous) with the variant that allocates them
# plainly (TBGPU_NO_CONTIG) and the timing-only no-flush variant (FP_NOFLUSH: results
# wrong by construction), fresh process each, same box.
OUT=${1:-gpurun_out/r03_drift}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', round(d['value']/1e9,3), r['dominant_ms_per_step'])" || true
  return $rc
}
ARGS="python3 bench.py --steps 8 --warmup 3 --no-cpu --no-queries --no-host"
V=tigerbeetle_amd/build
run p1 TB_X=1 $ARGS &&
run c1 TBGPU_LIB=$V/var_nocontig/libtbgpu.so $ARGS &&
run n1 TBGPU_LIB=$V/var_noflush/libtbgpu.so $ARGS &&
run p2 TB_X=1 $ARGS &&
run c2 TBGPU_LIB=$V/var_nocontig/libtbgpu.so $ARGS &&
run n2 TBGPU_LIB=$V/var_noflush/libtbgpu.so $ARGS &&
run p3 TB_X=1 $ARGS &&
run c3 TBGPU_LIB=$V/var_nocontig/libtbgpu.so $ARGS
