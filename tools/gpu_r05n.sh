# round-5 evidence: config-3 kernel summary, PMC traffic, SQ counters of the main kernels, config-1
# kernel summary, the prefilter microbenchmark, and config 5 (PMC table of the warm step, then the
# bench line reading it, then the kernel summary of the same command's warm step)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/profile.sh kernels r05c3 > gpurun_out/r05n_k3.log 2>&1 || { tail -5 gpurun_out/r05n_k3.log; exit 1; }
head -14 gpurun_out/prof_r05c3.txt
bash tools/profile.sh traffic r05 > gpurun_out/r05n_tr.log 2>&1 || { tail -5 gpurun_out/r05n_tr.log; exit 2; }
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_traffic_r05.json')); print({k: round(v['bytes']/1e6,1) for k,v in d['stages'].items()}, round(sum(v['bytes'] for v in d['stages'].values())/1e6,1))"
bash tools/profile.sh sq "bucket_small|pt_scatter_capped|pt_reduce_fast|bp_scatter2g|bp_scatter1p" r05 > gpurun_out/r05n_sq.log 2>&1 || { tail -5 gpurun_out/r05n_sq.log; exit 3; }
cat gpurun_out/sq_r05.txt | head -12
bash tools/profile.sh kernels r05c1 --config config1 > gpurun_out/r05n_k1.log 2>&1 || { tail -5 gpurun_out/r05n_k1.log; exit 4; }
head -14 gpurun_out/prof_r05c1.txt
timeout -k 10 60 ./tools/prefilter_bench > gpurun_out/prefilter_r05n.txt 2>&1 || exit 5
cat gpurun_out/prefilter_r05n.txt
bash tools/profile.sh traffic5 r05 > gpurun_out/r05n_tr5.log 2>&1 || { tail -5 gpurun_out/r05n_tr5.log; exit 6; }
cp gpurun_out/pmc_config5_r05.json profiles/r05_pmc_config5.json
timeout -k 10 500 python3 bench.py --config config5 --warmup 1 > gpurun_out/r05n_bench_config5.json 2> gpurun_out/r05n_bench_config5.err || exit 7
python3 -c "
import json; d=json.load(open('gpurun_out/r05n_bench_config5.json')); r=d['roofline']; print('config5', round(d['ms_per_step'],1), d['config']['passes'], r['traffic'], r.get('traffic_source'), d.get('digest'))"
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf gpurun_out/prof_r05c5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05c5 -o run -- python3 bench.py --config config5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r05c5.json 2> gpurun_out/prof_r05c5.err || exit 8
python3 tools/trace_after_marker.py $(find gpurun_out/prof_r05c5 -name 'run_kernel_trace.csv') > gpurun_out/prof_r05c5.txt
head -16 gpurun_out/prof_r05c5.txt
rm -f $(find gpurun_out/prof_r05c5 -name 'run_kernel_trace.csv')
