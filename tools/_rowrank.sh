set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rowsort.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/rowsort_tests.log 2>&1 || { tail -40 gpurun_out/rowsort_tests.log; exit 1; }
tail -3 gpurun_out/rowsort_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_rank.json 2> gpurun_out/bench_rank.err
KMP_PT_RANK=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_radix.json 2> gpurun_out/bench_radix.err
python - <<'PY'
import json
for f in ("gpurun_out/bench_rank.json", "gpurun_out/bench_radix.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 4), {k: round(v["ms"], 4) for k, v in d["roofline"]["stages"].items()}, d["config"]["edges"])
PY
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rank -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_rank.json 2> gpurun_out/prof_rank.err
echo profiled
