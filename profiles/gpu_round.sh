set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && tail -3 gpurun_out/gpu_tests.log && \
timeout -k 10 180 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json && \
bash profiles/collect.sh gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1; echo collect=$?; tail -40 gpurun_out/pmc_summary.txt
