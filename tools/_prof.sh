# kernel-trace profile of the default bench (no CPU baseline) -> gpurun_out/prof_<tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err
python tools/prof_summary.py $(find gpurun_out/prof_$TAG -name 'run_kernel_stats.csv' | head -1) 24
