set -o pipefail
O=gpurun_out/d3; mkdir -p $O
TBGPU_TRACE_PASSES=1 timeout -k 10 200 python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-queries --no-subconfigs --no-host > $O/trace.json 2> $O/trace.err || exit 1
TBGPU_EVAL_PROBE=1 timeout -k 10 200 python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-queries --no-subconfigs --no-host > $O/probe.json 2> $O/probe.err || exit 2
