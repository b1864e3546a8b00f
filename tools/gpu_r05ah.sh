# hot-file tidy (decided A/B alternatives removed): parity and multi tests, one config-3 and config-1 line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_dist.py -m gpu > gpurun_out/r05ah_tests.log 2>&1 || { tail -20 gpurun_out/r05ah_tests.log; exit 1; }
tail -1 gpurun_out/r05ah_tests.log
for c in config3 config1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/r05ah_$c.json 2> gpurun_out/r05ah_$c.err || exit 2
  python3 -c "
import json; d=json.load(open('gpurun_out/r05ah_$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in r['stages'].items()})"
done
