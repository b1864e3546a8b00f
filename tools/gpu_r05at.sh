# A/B: fast-tail row blocks of ~1,100 keys (ft1100) against ~2,275 (base): config 3, then G = 8 per rank (emulated)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/ft1100/libkmerpair.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/r05at_tests.log 2>&1 || { tail -20 gpurun_out/r05at_tests.log; exit 1; }
tail -1 gpurun_out/r05at_tests.log
CONFIGS="config3" timeout -k 10 600 bash tools/ab_multi.sh || exit 2
for v in base ft1100; do
  if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/$v/libkmerpair.so; fi
  timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 8 > gpurun_out/r05at_dist_$v.txt 2>&1 || exit 3
  echo $v; grep "^8 wall" gpurun_out/r05at_dist_$v.txt
done
