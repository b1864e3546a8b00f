# the overlapped front (level 2 + bucket kernels on two streams): the GPU suite, then the A/B
# against the one-stream front (noovl) on configs 3 and 1, then the per-rank split timing
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_r05p.log 2>&1; rc=$?
tail -2 gpurun_out/tests_r05p.log
grep -E "FAILED|Error" gpurun_out/tests_r05p.log | head -5
if [ $rc -ne 0 ]; then exit $rc; fi
CONFIGS="config3 config1" timeout -k 10 600 bash tools/ab_multi.sh > gpurun_out/ab_r05p.txt 2>&1 || { cat gpurun_out/ab_r05p.txt; exit 2; }
cat gpurun_out/ab_r05p.txt
timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 2 4 8 > gpurun_out/dist_sharded_r05p.txt 2>&1 || exit 3
head -5 gpurun_out/dist_sharded_r05p.txt
