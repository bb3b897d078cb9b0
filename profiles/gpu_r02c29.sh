#!/bin/bash
# the drop-in call's timeline (kernel trace of 64 single-batch calls)
set -o pipefail
O=gpurun_out/r02c29; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u profiles/single_call.py 64 > $O/plain.txt 2>&1; echo "plain rc=$?"; tail -1 $O/plain.txt
timeout -s KILL 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt -o kt --output-format csv -- python3 profiles/single_call.py 64 > $O/kt.log 2>&1; echo "kt rc=$?"; grep "single call" $O/kt.log
