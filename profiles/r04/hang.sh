#!/bin/bash
# the config-3 checkpoint test that stopped: this build (traced), then the previous commit's build
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
T="tests/test_gpu_checkpoint.py::test_checkpoint_restore_continue[3]"
TBGPU_LIB=$PWD/tigerbeetle_amd/build/var_prev/libtbgpu.so timeout -k 10 120 python3 -u -m pytest -x -q -s --timeout 90 --timeout-method thread "$T" > $O/prev.txt 2>&1
echo "prev rc=$?" >> $O/prev.txt
TBGPU_TRACE_PASSES=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 120 python3 -u -m pytest -x -q -s --timeout 90 --timeout-method thread "$T" > $O/cur.txt 2>&1
echo "cur rc=$?" >> $O/cur.txt
