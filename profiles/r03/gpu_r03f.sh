#!/bin/bash
# Round 3: the walk's mismatch on test_walk_matches_the_passes[config3] (r03e) -- four
# runs of the same workload, first differing events.
OUT=gpurun_out/r03f
mkdir -p "$OUT"
timeout -k 10 300 python3 -u profiles/r03/debug_walk.py > "$OUT/debug_walk.txt" 2>&1
rc=$?; cat "$OUT/debug_walk.txt" | grep -v amdgpu.ids; exit $rc
