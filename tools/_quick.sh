# selected GPU tests (PYTEST_K) then the config-3 bench line (no CPU baseline) and its kernel stats
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "${PYTEST_K:-partitions}" > gpurun_out/quick_tests.log 2>&1 || { tail -40 gpurun_out/quick_tests.log; exit 1; }
tail -3 gpurun_out/quick_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err
python -c "
import json; d=json.load(open('gpurun_out/quick_bench.json')); r=d['roofline']
print('ms/step', round(d['ms_per_step'],4), 'frac', round(r['frac'],3), {k: round(v['ms'],4) for k,v in r['stages'].items()})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_quick -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_quick.json 2> gpurun_out/prof_quick.err
python tools/prof_summary.py $(find gpurun_out/prof_quick -name 'run_kernel_stats.csv') 16
