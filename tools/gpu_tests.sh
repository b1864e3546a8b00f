# GPU tests selected by $PYTEST_K (default: all) + optional bench line, logs under gpurun_out/
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_FILES:-tests} > gpurun_out/tests_$TAG.log 2>&1 || { tail -80 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  python -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json')); r=d['roofline']
print('ms/step', round(d['ms_per_step'],4), 'frac', round(r['frac'],3), {k: round(v['ms'],4) for k,v in r['stages'].items()})"
fi
