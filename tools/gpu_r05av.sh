# A/B: level 1 at 1,024 threads of 4 slots (l1t1024) against 512 of 8 (base): parity of the variant, configs 3 and 1, G = 8 per rank
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/l1t1024/libkmerpair.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/r05av_tests.log 2>&1 || { tail -20 gpurun_out/r05av_tests.log; exit 1; }
tail -1 gpurun_out/r05av_tests.log
CONFIGS="config3 config1" timeout -k 10 600 bash tools/ab_multi.sh || exit 2
for v in base l1t1024; do
  if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/$v/libkmerpair.so; fi
  timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 8 > gpurun_out/r05av_dist_$v.txt 2>&1 || exit 3
  echo $v; grep "^8 wall" gpurun_out/r05av_dist_$v.txt
done
