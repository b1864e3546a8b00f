# spill-cursor copy by a kernel: parity, config 1 three lines, config-1 kernel trace (gaps)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu > gpurun_out/r05am_tests.log 2>&1 || { tail -20 gpurun_out/r05am_tests.log; exit 1; }
tail -1 gpurun_out/r05am_tests.log
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --config config1 --steps 40 > gpurun_out/r05am_c1.json 2>/dev/null || exit 2
  python3 -c "
import json; d=json.load(open('gpurun_out/r05am_c1.json')); print('config1', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in d['roofline']['stages'].items()})"
done
bash tools/profile.sh kernels r05am1 --config config1 > gpurun_out/r05am_k1.log 2>&1 || exit 3
