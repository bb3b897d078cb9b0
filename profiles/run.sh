#!/bin/bash
# The one runner for the GPU evidence under profiles/ (run on the GPU box from the
# repo root, e.g. gpurun -- bash profiles/run.sh gpurun_out/r05a suite smoke driver):
#
#   bash profiles/run.sh OUT STEP [STEP ...]
#
#   suite               pytest -m gpu, one process                       OUT/gpu_tests.txt
#   smoke               __graft_entry__.smoke()                          OUT/smoke.txt
#   driver[:K]          the driver's command, K times (default 1)        OUT/bench[.k].json
#   config:C[:A,B..]    bench.py --config C plus arguments A B ..        OUT/bench_configC[_tag].json
#                       (commas stand for spaces: config:1:--id-order,random)
#   pmc:C[:ORDER]       kernel trace + PMC passes of config C's bench    OUT/pmcC[_ORDER]/ (+ traffic.json)
#                       step (profiles/collect.sh), ids in ORDER; pmc:4:routed: the routed step
#                       on a one-rank group                              OUT/pmc4_routed/
#   hostpath            the drop-in call's kernel timeline               OUT/hostpath/
#   fuzz:FIRST:COUNT[:big|:random]  the on-demand fuzz sweep (full-size batches, or
#                       random u128 ids)                                 OUT/fuzz_FIRST[MODE].txt
#   passes:C            pass trace of config C (TBGPU_TRACE_PASSES=1)    OUT/passes_configC.json
#   ab:V1,V2[:A,B..]    timing variants (profiles/variants.py; `base` is the product library,
#                       others build/var_NAME built beforehand), REPS alternations
#                                                                        OUT/ab_V1_V2.txt
#
# Every step has its own time limit; the first step that fails ends the run (no step
# runs on the GPU after a fault, an abort or a timeout).  TBGPU_* variables pass
# through to every step (A/B runs of the engine's switches).
set -o pipefail
OUT=${1:?usage: run.sh OUT STEP...}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
Q="--no-cpu --no-queries --no-subconfigs --no-host"

accounts_of() { case $1 in 1|3) echo 10000;; 2) echo 1000000;; 4) echo 10000000;; 5) echo 100000000;; esac; }
events_of() { case $1 in 3) echo 491400;; *) echo 8190000;; esac; }

step() {
  local s=$1 kind rest
  kind=${s%%:*}; rest=${s#*:}; [ "$rest" = "$s" ] && rest=""
  echo "[run.sh] $(date +%T) $s" >&2
  case $kind in
    suite)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/gpu_tests.txt" 2>&1 ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 ;;
    driver)
      local k n=${rest:-1}
      for k in $(seq 1 "$n"); do
        local f=$OUT/bench.json; [ "$n" -gt 1 ] && f=$OUT/bench.$k.json
        timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$f" 2> "${f%.json}.err" || return 1
      done ;;
    config)
      local c=${rest%%:*} a="" tag=""
      [ "$rest" != "$c" ] && a=${rest#*:} && tag=_$(echo "$a" | tr -c 'a-z0-9\n' '_' | tr -s _)
      timeout -k 10 600 python3 -u bench.py --config "$c" ${a//,/ } > "$OUT/bench_config$c$tag.json" \
        2> "$OUT/bench_config$c$tag.err" ;;
    pmc)
      local c=${rest%%:*} order=sequential routed="" extra=""
      [ "$rest" != "$c" ] && order=${rest#*:}
      # pmc:4:routed profiles the routed step on a one-rank group (the scaling family's N = 1)
      [ "$order" = routed ] && { order=sequential; routed=1; extra="--routed"; }
      local d=$OUT/pmc$c; [ "$order" != sequential ] && d=${d}_$order; [ -n "$routed" ] && d=${d}_routed
      local steps="--steps 2 --warmup 1"
      TB_CONFIG=$c TB_ACCOUNTS=$(accounts_of "$c") TB_CALLS=3 TB_ID_ORDER=$order TB_ROUTED=$routed \
        EVENTS_PER_LAUNCH=$(events_of "$c") \
        bash profiles/collect.sh "$d" --config "$c" --id-order "$order" $extra $steps $Q > "$d.log" 2>&1 ;;
    hostpath)
      mkdir -p "$OUT/hostpath"
      timeout -k 10 300 python3 -u profiles/hostpath_trace.py > "$OUT/hostpath/plain.txt" 2>&1 || return 1
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/hostpath/kt" -o kt --output-format csv -- \
        python3 -u "$ROOT/profiles/hostpath_trace.py" > "$ROOT/$OUT/hostpath/kt.log" 2>&1) ;;
    fuzz)
      local first=${rest%%:*} r2=${rest#*:} count mode="" big="" rnd=""
      count=${r2%%:*}; [ "$r2" != "$count" ] && mode=${r2#*:}
      case $mode in big) big=1;; random) rnd=1;; esac
      TB_FUZZ_BIG=$big TB_FUZZ_RANDOM=$rnd TB_FUZZ_STRESS=$first:$count timeout -k 10 900 python3 -u -m pytest -x -q -s \
        --timeout 880 --timeout-method thread tests/test_gpu_fuzz.py -k stress > "$OUT/fuzz_$first$mode.txt" 2>&1 ;;
    passes)
      TBGPU_TRACE_PASSES=1 timeout -k 10 300 python3 -u bench.py --config "$rest" --steps 1 --warmup 0 $Q \
        > "$OUT/passes_config$rest.json" 2> "$OUT/passes_config$rest.err" ;;
    ab)
      local v=${rest%%:*} a="--steps 5 --warmup 1 $Q"
      [ "$rest" != "$v" ] && a=${rest#*:} && a="${a//,/ } $Q"
      timeout -k 10 900 python3 -u profiles/variants.py ${v//,/ } -- $a > "$OUT/ab_${v//,/_}.txt" 2>&1 ;;
    *)
      echo "run.sh: unknown step $s" >&2; return 2 ;;
  esac
}

for s in "$@"; do
  step "$s" || { rc=$?; echo "[run.sh] step $s failed ($rc): stopping" >&2; exit $rc; }
done
echo "[run.sh] done" >&2
