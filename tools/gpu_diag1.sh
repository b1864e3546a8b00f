# diagnostic: the two-process bench path (residue start) with serialised kernels and the library's
# launch trace, output uncaptured
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
KMP_TRACE=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 240 python -u -m pytest tests/test_gpu_dist.py -k bench_multi -x -s --timeout 200 --timeout-method thread > gpurun_out/diag1.log 2>&1; rc=$?
grep -v "^frame" gpurun_out/diag1.log | tail -60
exit $rc
