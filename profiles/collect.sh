#!/bin/bash
# rocprofv3 recipe for the bench's kernels (run on the GPU box from the repo root):
# one kernel-trace/stats pass, then one pass per PMC group (rocprofv3 does not
# split counters over passes; FETCH_SIZE and WRITE_SIZE need separate passes).
#   TB_CONFIG=3 TB_ACCOUNTS=10000 TB_CALLS=3 EVENTS_PER_LAUNCH=491400 \
#   bash profiles/collect.sh OUTDIR [bench args...]
# TB_* tag traffic.json's _meta with the workload (bench.py's pmc_traffic matches on
# config + accounts); TB_CALLS = warmup + steps of the profiled command.
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:---steps 2 --warmup 1 --no-cpu --no-queries --no-subconfigs --no-host}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py $ARGS"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- $B > "$OUT/kt.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/p1" -o p1 --output-format csv -- $B > "$OUT/p1.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/p2" -o p2 --output-format csv -- $B > "$OUT/p2.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/p3" -o p3 --output-format csv -- $B > "$OUT/p3.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM -d "$OUT/p4" -o p4 --output-format csv -- $B > "$OUT/p4.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d "$OUT/p5" -o p5 --output-format csv -- $B > "$OUT/p5.log" 2>&1
python3 profiles/summarize.py "$OUT" ${EVENTS_PER_LAUNCH:-8190000} "$OUT/traffic.json"
