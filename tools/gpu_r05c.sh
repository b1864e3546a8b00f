cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_r05f.log 2>&1; rc=$?
tail -25 gpurun_out/tests_r05f.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 2 4 8 > gpurun_out/dist_sharded_r05f.txt 2>&1
rc=$?; head -5 gpurun_out/dist_sharded_r05f.txt; [ $rc -ne 0 ] && exit $rc
TAG=r05f MODE=sharded bash tools/prof_split.sh config3 8 2>&1 | head -22
