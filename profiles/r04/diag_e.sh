# Round 4 diagnosis: the order-dependent failures under memory / coherence variants,
# each suite stopping at its first failure (its details printed).
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT; export TMPDIR=/tmp; export TBGPU_FATAL_LOG=$PWD/$OUT/fatal.log
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests -m gpu"
for v in default nocontig flush nosdma; do
  case $v in
    default) E="TBGPU_UNUSED=1" ;;
    nocontig) E="TBGPU_NO_CONTIG=1" ;;
    flush) E="TBGPU_FLUSH_CALLS=1" ;;
    nosdma) E="HSA_ENABLE_SDMA=0" ;;
  esac
  timeout -k 10 400 env $E $PT > $OUT/$v.txt 2>&1
  rc=$?
  echo "$v rc=$rc: $(grep -c PASSED $OUT/$v.txt) passed; $(grep -m1 FAILED $OUT/$v.txt)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
