# config-1 bench line (no CPU baseline) and its kernel stats
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_c1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1 -o run -- python3 bench.py --config config1 --no-cpu-baseline > gpurun_out/prof_c1.json 2> gpurun_out/prof_c1.err
timeout -k 10 300 python bench.py --config config1 --no-cpu-baseline > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err
python -c "
import json; d=json.load(open('gpurun_out/bench_c1.json')); r=d['roofline']
print('config1 ms/step', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in r['stages'].items()})"
python tools/prof_summary.py $(find gpurun_out/prof_c1 -name 'run_kernel_stats.csv' | head -1) 30
