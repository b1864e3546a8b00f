# config-1 kernel stats for each KMP_LIB variant given (abvar/<name>.so), 8 steps each
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  rm -rf gpurun_out/abc1_$v
  KMP_LIB=abvar/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abc1_$v -o run -- python3 bench.py --config config1 --no-cpu-baseline --steps 8 --warmup 2 > gpurun_out/abc1_$v.json 2> gpurun_out/abc1_$v.err
  echo "== $v"; python3 -c "import json; print('ms/step', json.load(open('gpurun_out/abc1_$v.json'))['ms_per_step'])"
  python tools/prof_summary.py $(find gpurun_out/abc1_$v -name 'run_kernel_stats.csv') 10 | head -8
done
