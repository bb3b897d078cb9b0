#!/bin/bash
# r02c evidence (third session of round 2): GPU tests, smoke, the driver's bench
# command, configs 1/3 (verify)/4/5, routed one-rank (plain and pipelined), a
# two-rank routed rehearsal (gloo collectives, both ranks on the one GPU), kernel
# traces and PMC passes of configs 2 and 4
set -o pipefail
O=gpurun_out/r02c_final8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.txt
timeout -k 10 200 python3 -u profiles/single_call.py 256 > $O/single_call.txt 2>&1; echo "single rc=$?"; tail -1 $O/single_call.txt
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; echo "bench rc=$? $(grep -o '"value": [0-9.]*' $O/bench.json | head -1) $(grep -o '"frac": [0-9.]*' $O/bench.json | head -1)"
timeout -k 10 300 python3 -u bench.py --config 1 --no-queries > $O/bench_config1.json 2> $O/bench_config1.err; echo "c1 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config1.json | head -1)"
timeout -k 10 300 python3 -u bench.py --config 3 --no-queries --verify > $O/bench_config3.json 2> $O/bench_config3.err; echo "c3 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config3.json | head -1)"
timeout -k 10 300 python3 -u bench.py --config 4 --no-queries > $O/bench_config4.json 2> $O/bench_config4.err; echo "c4 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config4.json | head -1)"
timeout -k 10 600 python3 -u bench.py --config 5 --no-queries > $O/bench_config5.json 2> $O/bench_config5.err; echo "c5 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_config5.json | head -1)"
timeout -k 10 400 python3 -u bench.py --routed --steps 6 --no-cpu > $O/bench_routed_1rank.json 2> $O/bench_routed_1rank.err; echo "routed rc=$? $(grep -o '"value": [0-9.]*' $O/bench_routed_1rank.json)"
timeout -k 10 400 python3 -u bench.py --routed --pipelined --steps 6 --no-cpu > $O/bench_routed_1rank_pipelined.json 2> $O/bench_routed_1rank_pipelined.err; echo "routed pipelined rc=$? $(grep -o '"value": [0-9.]*' $O/bench_routed_1rank_pipelined.json)"
TB_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --batches-per-step 100 > $O/bench_routed_gloo2.json 2> $O/bench_routed_gloo2.err; echo "gloo2 rc=$? $(grep -o '"value": [0-9.]*' $O/bench_routed_gloo2.json)"
TB_CONFIG=2 TB_ACCOUNTS=1000000 TB_CALLS=3 bash profiles/collect.sh $O/c2 --config 2 --steps 2 --warmup 1 --no-cpu --no-queries --no-host && python3 profiles/summarize.py $O/c2 8190000 > $O/c2/summary.txt && echo c2 pmc ok
TB_CONFIG=3 TB_ACCOUNTS=10000 TB_CALLS=3 EVENTS_PER_LAUNCH=491400 bash profiles/collect.sh $O/c3 --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host && python3 profiles/summarize.py $O/c3 491400 > $O/c3/summary.txt && echo c3 pmc ok
TB_CONFIG=4 TB_ACCOUNTS=10000000 TB_CALLS=3 bash profiles/collect.sh $O/c4 --config 4 --steps 2 --warmup 1 --no-cpu --no-queries --no-host && python3 profiles/summarize.py $O/c4 8190000 > $O/c4/summary.txt && echo c4 pmc ok
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_routed -o kt --output-format csv -- python3 bench.py --routed --steps 2 --no-cpu > $O/kt_routed.log 2>&1 && echo routed kt ok
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_c3 -o kt --output-format csv -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu --no-queries --no-host > $O/kt_c3.log 2>&1 && echo c3 kt ok
