# One parameterised GPU runner for round 4 (replaces the one-off gpu_r03*/final_*/diag_* scripts).
#   bash profiles/r04/run.sh OUT STEP [STEP...]
# Steps: suite | suite_x | poison_queries | poison_suite | smoke | bench | bench_cfg<N> | prof_cfg<N> | pytest:<args>
# Every GPU step runs under its own timeout; the first failing step ends the script.
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
export TBGPU_FATAL_LOG=$PWD/$OUT/fatal.log
PT="python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider"
run() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.txt" 2>&1
    local rc=$?
    tail -3 "$OUT/$name.txt"
    echo "== $name rc=$rc"
    return $rc
}
ok1() {  # a suite whose tests failed (pytest rc 1) lets the next step run; anything else ends the script
    local rc=$?
    [ $rc -eq 1 ] || exit 1
}
for step in "$@"; do
    case $step in
    suite) run suite 600 $PT tests -m gpu || ok1 ;;
    suite_x) run suite_x 600 $PT -x tests -m gpu || exit 1 ;;
    poison_queries) run poison_queries 300 env TBGPU_POISON_ALLOC=1 TBGPU_CHECK_INDEX=1 $PT tests/test_gpu_queries.py || exit 1 ;;
    poison_suite) run poison_suite 700 env TBGPU_POISON_ALLOC=1 TBGPU_CHECK_INDEX=1 $PT tests -m gpu || ok1 ;;
    sdma_suite) run sdma_suite 600 env TBGPU_SDMA_H2D=1 $PT tests -m gpu || ok1 ;;
    sdma_off_suite) run sdma_off_suite 600 env TBGPU_SDMA_H2D=1 HSA_ENABLE_SDMA=0 $PT tests -m gpu || ok1 ;;
    nocontig_suite) run nocontig_suite 600 env TBGPU_NO_CONTIG=1 $PT tests -m gpu || ok1 ;;
    flush_suite) run flush_suite 600 env TBGPU_FLUSH_CALLS=1 $PT tests -m gpu || ok1 ;;
    nosdma_suite) run nosdma_suite 600 env HSA_ENABLE_SDMA=0 $PT tests -m gpu || ok1 ;;
    smoke) run smoke 180 python -u __graft_entry__.py smoke || exit 1 ;;
    bench) run bench 400 python bench.py || exit 1 ;;
    bench_cfg*) run "bench_cfg${step#bench_cfg}" 400 python bench.py --config "${step#bench_cfg}" || exit 1 ;;
    pytest:*) run "pytest_$(echo "${step#pytest:}" | tr -c 'A-Za-z0-9' _ | cut -c1-60)" 600 $PT ${step#pytest:} || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
