# config-5 bench line (k = 7, 1M proteins, BLOSUM, with the CPU baseline) and its kernel stats
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config config5 --steps 2 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config config5 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/prof_c5.json 2> gpurun_out/prof_c5.err
python tools/prof_summary.py $(find gpurun_out/prof_c5 -name 'run_kernel_stats.csv' | head -1) 20 > gpurun_out/summary_c5.txt
