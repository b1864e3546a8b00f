# diagnostic: the two-process bench path (residue start) with the library's launch trace and
# host-side checks of the routed keys after every expand and before every edges call
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
KMP_TRACE=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_dist.py -k bench_multi -x -s --timeout 200 --timeout-method thread > gpurun_out/diag2.log 2>&1; rc=$?
grep -E "kmp-trace: split_(expand part|edges received)|Error|error|PASS|FAIL|passed|failed" gpurun_out/diag2.log | head -60
exit $rc
