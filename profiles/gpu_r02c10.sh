#!/bin/bash
# routed one-rank step under cProfile: where the host time goes
set -o pipefail
O=gpurun_out/r02c10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m cProfile -o $O/routed.prof bench.py --routed --steps 6 --no-cpu > $O/routed.json 2> $O/routed.err; echo "routed rc=$?"
python3 -c "
import pstats; p = pstats.Stats('$O/routed.prof'); p.sort_stats('tottime').print_stats(40)" > $O/prof.txt 2>&1; echo done
