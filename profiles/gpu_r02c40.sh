#!/bin/bash
# fp_commit leaves an HBM copy of in-place (host) events for the later launches:
# GPU suite, single-call A/B, config-4 host_path (chains), config-2 bench
set -o pipefail
O=gpurun_out/r02c40; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  timeout -k 10 200 python3 -u profiles/single_call.py 256 > $O/zc_$r.txt 2>&1 || exit 1; tail -1 $O/zc_$r.txt
  TBGPU_NO_ZERO_COPY=1 timeout -k 10 200 python3 -u profiles/single_call.py 256 > $O/copy_$r.txt 2>&1 || exit 1; tail -1 $O/copy_$r.txt
done
for v in zc copy; do
  E=""; [ $v = copy ] && E="TBGPU_NO_ZERO_COPY=1"
  env $E timeout -k 10 300 python3 -u bench.py --config 4 --no-queries --no-cpu --steps 2 > $O/c4_$v.json 2> $O/c4_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/c4_$v.json').read().strip().splitlines()[-1]); print('c4 $v', d['value']/1e9, d['host_path']['single']['latency_us'])"
done
timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-queries > $O/c2.json 2> $O/c2.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); print('c2', d['value']/1e9, d['roofline']['frac'], d['host_path']['single']['latency_us'])"
