# config-5 evidence on the final tree: PMC table of the warm step, the bench line (with its CPU baseline sample)
# reading it, and the kernel summary of the same command's warm step
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/profile.sh traffic5 r05f > gpurun_out/r05ax_tr5.log 2>&1 || { tail -5 gpurun_out/r05ax_tr5.log; exit 1; }
cp gpurun_out/pmc_config5_r05f.json profiles/r05_pmc_config5.json
timeout -k 10 500 python3 bench.py --config config5 --warmup 1 > gpurun_out/r05ax_bench_config5.json 2> gpurun_out/r05ax_bench_config5.err || exit 2
python3 -c "
import json; d=json.load(open('gpurun_out/r05ax_bench_config5.json')); r=d['roofline']; print('config5', round(d['ms_per_step'],1), d['config']['passes'], r['traffic'], r.get('traffic_source'), d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf gpurun_out/prof_r05fc5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05fc5 -o run -- python3 bench.py --config config5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r05fc5.json 2> gpurun_out/prof_r05fc5.err || exit 3
python3 tools/trace_after_marker.py $(find gpurun_out/prof_r05fc5 -name 'run_kernel_trace.csv') > gpurun_out/prof_r05fc5.txt
head -16 gpurun_out/prof_r05fc5.txt
rm -f $(find gpurun_out/prof_r05fc5 -name 'run_kernel_trace.csv')
