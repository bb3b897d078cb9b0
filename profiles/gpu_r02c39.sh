#!/bin/bash
# events read in place from pinned host memory for small one-chunk calls: GPU suite,
# then the drop-in call A/B against the copy (TBGPU_NO_ZERO_COPY=1), then its timeline
set -o pipefail
O=gpurun_out/r02c39; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  timeout -k 10 200 python3 -u profiles/single_call.py 256 > $O/zc_$r.txt 2>&1 || exit 1; tail -1 $O/zc_$r.txt
  TBGPU_NO_ZERO_COPY=1 timeout -k 10 200 python3 -u profiles/single_call.py 256 > $O/copy_$r.txt 2>&1 || exit 1; tail -1 $O/copy_$r.txt
done
timeout -s KILL 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt -o kt --output-format csv -- python3 profiles/single_call.py 64 > $O/kt.log 2>&1; echo "kt rc=$?"; grep "single call" $O/kt.log
