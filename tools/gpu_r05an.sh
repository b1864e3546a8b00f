# round-5 evidence on the final tree: the GPU test suite, bench
# lines (config 3 with its CPU baseline, configs 1, 2 and 5), kernel summaries (configs 3 and 1), PMC
# traffic and SQ counters, the sharded k-mer split per rank at G = 8 (emulated)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r05an_tests.log 2>&1 || { tail -20 gpurun_out/r05an_tests.log; exit 1; }
tail -1 gpurun_out/r05an_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r05an_bench_config3.json 2> gpurun_out/r05an_bench_config3.err || exit 2
python3 -c "
import json; d=json.load(open('gpurun_out/r05an_bench_config3.json')); r=d['roofline']; print('config3', round(d['ms_per_step'],4), r['frac'], r['traffic'], d['cpu_baseline']['value'], {k: round(v['ms'],4) for k,v in r['stages'].items()})"
for c in config1 config2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/r05an_bench_$c.json 2> gpurun_out/r05an_bench_$c.err || exit 3
  python3 -c "
import json; d=json.load(open('gpurun_out/r05an_bench_$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in r['stages'].items()})"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --config config5 --warmup 1 > gpurun_out/r05an_bench_config5.json 2> gpurun_out/r05an_bench_config5.err || exit 4
python3 -c "
import json; d=json.load(open('gpurun_out/r05an_bench_config5.json')); print('config5', round(d['ms_per_step'],1))"
bash tools/profile.sh kernels r05an3 > gpurun_out/r05an_k3.log 2>&1 || exit 5
head -10 gpurun_out/prof_r05an3.txt
bash tools/profile.sh kernels r05an1 --config config1 > gpurun_out/r05an_k1.log 2>&1 || exit 6
head -10 gpurun_out/prof_r05an1.txt
bash tools/profile.sh traffic r05an > gpurun_out/r05an_tr.log 2>&1 || exit 7
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_traffic_r05an.json')); print({k: round(v['bytes']/1e6,1) for k,v in d['stages'].items()}, round(sum(v['bytes'] for v in d['stages'].values())/1e6,1))"
bash tools/profile.sh sq "bucket_small|pt_scatter_capped|pt_reduce_fast|bp_scatter2g|bp_scatter1p" r05an > gpurun_out/r05an_sq.log 2>&1 || exit 8
timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 8 > gpurun_out/r05an_dist8.txt 2>&1 || exit 9
tail -4 gpurun_out/r05an_dist8.txt
