#!/bin/bash
# Round 3, session 2, first GPU call: the driver's headline command as the FIRST GPU
# process on the lease (SMI clock samples beside it), the same again, then the whole
# -m gpu suite and smoke().
OUT=gpurun_out/r03b
mkdir -p "$OUT"
( while true; do
    echo "=== $(date +%s.%N)"
    timeout 10 rocm-smi --showclocks --showpower --showtemp --json 2>&1 | head -c 4000
    sleep 2
  done ) > "$OUT/smi.log" 2>&1 &
SMI=$!
trap 'kill $SMI 2>/dev/null' EXIT
echo "== driver start $(date +%s.%N)" >> "$OUT/smi.log"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver.json" 2> "$OUT/driver.err" || exit $?
echo "== driver end $(date +%s.%N)" >> "$OUT/smi.log"
python3 profiles/r03/line.py "$OUT/driver.json"
echo "== second start $(date +%s.%N)" >> "$OUT/smi.log"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-queries --no-host > "$OUT/second.json" 2> "$OUT/second.err" || exit $?
echo "== second end $(date +%s.%N)" >> "$OUT/smi.log"
python3 profiles/r03/line.py "$OUT/second.json"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 || { tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 120 python3 __graft_entry__.py smoke > "$OUT/smoke.txt" 2>&1 || exit $?
cat "$OUT/smoke.txt"
