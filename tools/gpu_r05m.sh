# the GPU suite, config 3 / 1 benches, per-rank timing, the prefilter microbenchmark and the
# config-5 pass-budget A/B (budget per call vs cached per batch)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_r05m.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r05m.log
grep -E "FAILED|Error" gpurun_out/tests_r05m.log | head -5
if [ $rc -ne 0 ]; then exit $rc; fi
for c in config3 config1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/r05m_bench_$c.json 2> gpurun_out/r05m_bench_$c.err || exit 3
  python3 -c "
import json; d=json.load(open('gpurun_out/r05m_bench_$c.json')); r=d['roofline']
print('$c', round(d['ms_per_step'],4), r['tail'], {k: round(v['ms'],4) for k,v in r['stages'].items()})"
done
timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 2 4 8 > gpurun_out/dist_sharded_r05m.txt 2>&1 || exit 4
head -5 gpurun_out/dist_sharded_r05m.txt
timeout -k 10 60 ./tools/prefilter_bench > gpurun_out/prefilter_r05m.txt 2>&1 || exit 5
cat gpurun_out/prefilter_r05m.txt
for v in cached percall; do
  if [ $v = percall ]; then export KMP_BUDGET_PER_CALL=1; fi
  timeout -k 10 400 python bench.py --config config5 --no-cpu-baseline --warmup 1 --steps 1 > gpurun_out/r05m_c5_$v.json 2> gpurun_out/r05m_c5_$v.err || exit 6
  python3 -c "
import json; d=json.load(open('gpurun_out/r05m_c5_$v.json')); print('$v', round(d['ms_per_step'],1), d['config']['passes'], d.get('digest'), {k: round(v['ms'],1) for k,v in d['roofline']['stages'].items()})"
done
