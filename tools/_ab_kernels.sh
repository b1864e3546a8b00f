# kernel stats of the config-3 step for each KMP_LIB variant given (abvar/<name>.so: a build of the
# library with changed kernels, copied there by hand), 8 steps each
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  rm -rf gpurun_out/ab_$v
  KMP_LIB=abvar/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$v -o run -- python3 bench.py --no-cpu-baseline --steps 8 --warmup 2 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  echo "== $v"; python tools/prof_summary.py $(find gpurun_out/ab_$v -name 'run_kernel_stats.csv') 4
done
