# GPU tests, then a kernel-trace profile of the default bench -> gpurun_out/prof_<tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-cur}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/_prof.sh $TAG
python -c "
import json; d = json.loads(open('gpurun_out/prof_$TAG.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], {k: round(v['ms'], 4) for k, v in d['roofline']['stages'].items()}, d['config']['edges'])"
