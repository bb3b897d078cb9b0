#!/bin/bash
set -o pipefail
O=gpurun_out/r02ad; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --routed --steps 2 --no-cpu > $O/routed.json 2> $O/routed.err; echo "rc=$? lines=$(grep -c '' $O/routed.json)"; python3 -c "import json;d=json.load(open('$O/routed.json'));print('json ok', d['value'])"
