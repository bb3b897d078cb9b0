#!/bin/bash
set -o pipefail
O=gpurun_out/r02w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --config 3 --verify --no-queries --no-host --no-cpu > $O/c3_verify.json 2> $O/c3_verify.err; echo "rc=$?"; grep -o '"verify": {[^}]*}' $O/c3_verify.json; grep -o '"value": [0-9.]*' $O/c3_verify.json
timeout -k 10 600 python3 -u bench.py --config 4 --steps 1 --verify --no-queries --no-host --no-cpu > $O/c4_verify.json 2> $O/c4_verify.err; echo "rc=$?"; grep -o '"verify": {[^}]*}' $O/c4_verify.json
