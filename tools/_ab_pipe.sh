set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for r in 1 2; do
for k in 1 2 4 8; do
KMP_PIPE=$k timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_pipe${k}_$r.json
done
done
python - <<'PY'
import json
for r in (1, 2):
    for k in (1, 2, 4, 8):
        f = f"gpurun_out/bench_pipe{k}_{r}.json"
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f, d["ms_per_step"], {k2: round(v["ms"], 4) for k2, v in d["roofline"]["stages"].items()}, d["config"]["edges"])
PY
