# bench ms/step (config 3, no profiler, no CPU baseline) for each KMP_LIB variant given, alternating
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "$@"; do
  KMP_LIB=abvar/$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/abb_$v.json 2> gpurun_out/abb_$v.err
  python3 -c "import json; print('$v', round(json.load(open('gpurun_out/abb_$v.json'))['ms_per_step'], 4))"
done
