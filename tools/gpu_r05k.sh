# the GPU suite on the current tree, then config 3 / config 1 benches and the per-rank timing
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_r05k.log 2>&1; rc=$?
tail -3 gpurun_out/tests_r05k.log
grep -E "FAILED|Error" gpurun_out/tests_r05k.log | head -5
if [ $rc -ne 0 ]; then exit $rc; fi
for c in config3 config1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/r05k_bench_$c.json 2> gpurun_out/r05k_bench_$c.err || exit 3
  python3 -c "
import json; d=json.load(open('gpurun_out/r05k_bench_$c.json')); r=d['roofline']
print('$c', round(d['ms_per_step'],4), r['tail'], {k: round(v['ms'],4) for k,v in r['stages'].items()})"
done
timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 2 4 8 > gpurun_out/dist_sharded_r05k.txt 2>&1
head -5 gpurun_out/dist_sharded_r05k.txt
