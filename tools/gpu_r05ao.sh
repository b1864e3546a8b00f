# the whole-bucket segment test, once with the segment histogram printed (KMP_TRACE)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
KMP_TRACE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "whole_bucket" -m gpu -s > gpurun_out/r05ao_tests.log 2>&1 || { tail -20 gpurun_out/r05ao_tests.log; exit 1; }
tail -1 gpurun_out/r05ao_tests.log
grep "segs" gpurun_out/r05ao_tests.log | sort | uniq -c | head
