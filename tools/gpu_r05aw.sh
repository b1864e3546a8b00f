# A/B: the counting tail's block sort on config 1 — radix (base), bin sort (bs2), radix with 4-bit digits (rb4); parity of bs2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/bs2/libkmerpair.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/r05aw_tests.log 2>&1 || { tail -20 gpurun_out/r05aw_tests.log; exit 1; }
tail -1 gpurun_out/r05aw_tests.log
CONFIGS="config1" timeout -k 10 600 bash tools/ab_multi.sh || exit 2
