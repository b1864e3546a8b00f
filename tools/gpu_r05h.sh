cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_multi.py -x -v --timeout 200 --timeout-method thread -k "device_stages or bench_multi or sharded" > gpurun_out/tests_r05h.log 2>&1; rc=$?
tail -15 gpurun_out/tests_r05h.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 2 4 8 > gpurun_out/dist_sharded_r05h.txt 2>&1
rc=$?; head -5 gpurun_out/dist_sharded_r05h.txt; exit $rc
