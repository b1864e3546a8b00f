cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 300 --timeout-method thread -k "sharded or routed" > gpurun_out/tests_r05c.log 2>&1; rc=$?
tail -15 gpurun_out/tests_r05c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 2 4 8 > gpurun_out/dist_sharded_r05c.txt 2>&1; rc2=$?
head -5 gpurun_out/dist_sharded_r05c.txt
exit $rc
