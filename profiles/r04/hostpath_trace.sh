#!/bin/bash
# kernel timeline of the drop-in call (profiles/r04/hostpath_trace.py)
set -o pipefail
O=gpurun_out/${TAG:-r04hp}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u profiles/r04/hostpath_trace.py > $O/plain.txt 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 -u $GRAFT_REPO_ROOT/profiles/r04/hostpath_trace.py > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 || exit 2
