# config3 + config1 bench lines, then a kernel-trace profile of each (no CPU baseline)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
cat gpurun_out/bench_c3.json
timeout -k 10 300 python bench.py --config config1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err
cat gpurun_out/bench_c1.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_c3.json 2> gpurun_out/prof_c3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1 -o run -- python3 bench.py --config config1 --no-cpu-baseline > gpurun_out/prof_c1.json 2> gpurun_out/prof_c1.err
python tools/prof_summary.py $(find gpurun_out/prof_c3 -name 'run_kernel_stats.csv' | head -1) 24
python tools/prof_summary.py $(find gpurun_out/prof_c1 -name 'run_kernel_stats.csv' | head -1) 30
