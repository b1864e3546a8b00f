# A/B: counting-tail partition tiles of 16,384 keys (base), 8,192 (pp8), 4,096 (pp4): parity of pp4 on the uniprot tail tests, config 1 and config 5
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/pp4/libkmerpair.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "uniprot or frequent or whole" -m gpu > gpurun_out/r05as_tests.log 2>&1 || { tail -20 gpurun_out/r05as_tests.log; exit 1; }
tail -1 gpurun_out/r05as_tests.log
CONFIGS="config1" timeout -k 10 600 bash tools/ab_multi.sh || exit 2
for v in base pp4; do
  if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/$v/libkmerpair.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --config config5 --warmup 1 > gpurun_out/r05as_c5_$v.json 2>/dev/null || exit 3
  python3 -c "
import json; d=json.load(open('gpurun_out/r05as_c5_$v.json')); print('config5 $v', round(d['ms_per_step'],1), {k: round(v['ms'],1) for k,v in d['roofline']['stages'].items()})"
done
