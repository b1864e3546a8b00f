# round-5 evidence on the current tree: bench lines (config 3 with its CPU baseline, configs 1 and 2),
# the config-3 kernel summary, PMC traffic and SQ counters, the config-1 kernel summary
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r05t_bench_config3.json 2> gpurun_out/r05t_bench_config3.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r05t_bench_config3.json')); r=d['roofline']; print('config3', round(d['ms_per_step'],4), r['frac'], r['traffic'], d['cpu_baseline']['value'], {k: round(v['ms'],4) for k,v in r['stages'].items()})"
for c in config1 config2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/r05t_bench_$c.json 2> gpurun_out/r05t_bench_$c.err || exit 2
  python3 -c "
import json; d=json.load(open('gpurun_out/r05t_bench_$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in r['stages'].items()})"
done
bash tools/profile.sh kernels r05t3 > gpurun_out/r05t_k3.log 2>&1 || exit 3
head -12 gpurun_out/prof_r05t3.txt
bash tools/profile.sh traffic r05t > gpurun_out/r05t_tr.log 2>&1 || exit 4
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_traffic_r05t.json')); print({k: round(v['bytes']/1e6,1) for k,v in d['stages'].items()}, round(sum(v['bytes'] for v in d['stages'].values())/1e6,1))"
bash tools/profile.sh sq "bucket_small|pt_scatter_capped|pt_reduce_fast|bp_scatter2g|bp_scatter1p" r05t > gpurun_out/r05t_sq.log 2>&1 || exit 5
head -7 gpurun_out/sq_r05t.txt
bash tools/profile.sh kernels r05t1 --config config1 > gpurun_out/r05t_k1.log 2>&1 || exit 6
head -8 gpurun_out/prof_r05t1.txt
