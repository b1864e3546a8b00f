# the fast reduce's look-back polling 4 words per lane per round: parity tests of the tails and the
# split, A/B against 1 word (lb1) on config 3, per-rank split timing
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r05s.log 2>&1; rc=$?
tail -2 gpurun_out/tests_r05s.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/tests_r05s.log | head -5; exit $rc; fi
timeout -k 10 600 bash tools/ab_multi.sh > gpurun_out/ab_r05s.txt 2>&1 || { cat gpurun_out/ab_r05s.txt; exit 2; }
cat gpurun_out/ab_r05s.txt
timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 2 4 8 > gpurun_out/dist_sharded_r05s.txt 2>&1 || exit 3
head -5 gpurun_out/dist_sharded_r05s.txt
for v in base lb1; do
  if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/$v/libkmerpair.so; fi
  timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 8 > gpurun_out/dist8_r05s_$v.txt 2>&1 || exit 4
  echo $v; sed -n 2,3p gpurun_out/dist8_r05s_$v.txt
done
