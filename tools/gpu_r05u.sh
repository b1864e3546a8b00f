# level 2's key -> run map by a block max-scan: parity (single-GPU and split paths), then an A/B against
# the per-thread fill loop on configs 3 and 1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu > gpurun_out/r05u_tests.log 2>&1 || { tail -20 gpurun_out/r05u_tests.log; exit 1; }
tail -2 gpurun_out/r05u_tests.log
CONFIGS="config3 config1" timeout -k 10 600 bash tools/ab_multi.sh || exit 2
