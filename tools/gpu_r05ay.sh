# the large segment sort forked before the spill-cursor copy (early=1, default) against after it (early=0): parity, config 1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu > gpurun_out/r05ay_tests.log 2>&1 || { tail -20 gpurun_out/r05ay_tests.log; exit 1; }
tail -1 gpurun_out/r05ay_tests.log
for i in 1 2 3; do
  for v in 1 0; do
    KMP_EARLY_FORK=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --config config1 --steps 40 > gpurun_out/ab_ef$v.json 2>/dev/null || exit 2
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_ef$v.json')); print('config1 early=$v', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in d['roofline']['stages'].items()})"
  done
done
