set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_part.json
KMP_PARTITION=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_sort.json
python - <<'PY'
import json
for f in ("gpurun_out/bench_part.json", "gpurun_out/bench_sort.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], {k: round(v["ms"], 4) for k, v in d["roofline"]["stages"].items()}, d["config"]["edges"])
PY
