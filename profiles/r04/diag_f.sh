# Round 4: the contiguous-allocation aliasing reproducer, then the suite and smoke on
# plain allocations, then the driver's bench command and a contiguous-allocation A/B.
set -o pipefail
OUT=gpurun_out/r04f; mkdir -p $OUT; export TMPDIR=/tmp; export TBGPU_FATAL_LOG=$PWD/$OUT/fatal.log
timeout -k 10 120 ./profiles/r04/contig_alias 40 > $OUT/contig_alias.txt 2>&1; echo "contig_alias rc=$? $(tail -1 $OUT/contig_alias.txt)"
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests -m gpu > $OUT/suite.txt 2>&1
rc=$?; echo "suite rc=$rc: $(tail -1 $OUT/suite.txt)"; grep FAILED $OUT/suite.txt | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u __graft_entry__.py smoke > $OUT/smoke.txt 2>&1 || exit 3
tail -1 $OUT/smoke.txt
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['value'], d['roofline']['frac'], {k:(v.get('value'),v.get('roofline',{}).get('frac')) for k,v in (d.get('configs') or {}).items()}, (d.get('scaling_n1') or {}).get('value'), d['create_accounts']['roofline']['frac'], d['host_path']['single']['latency_us'], d['host_path'].get('prefetched',{}).get('commit_latency_us'))"
timeout -k 10 300 env TBGPU_CONTIG=1 python bench.py --steps 5 --warmup 2 --no-subconfigs --no-cpu --no-host --no-queries > $OUT/bench_contig.json 2> $OUT/bench_contig.err
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-subconfigs --no-cpu --no-host --no-queries > $OUT/bench_plain.json 2> $OUT/bench_plain.err
python3 -c "
import json
for n in ('contig','plain'):
    d=json.load(open('$OUT/bench_'+n+'.json')); print(n, d['value'], d['roofline']['frac'], d['roofline']['dominant_ms_per_step'])"
