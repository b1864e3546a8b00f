# A/B of the tail variants (tools/ab) on config 3 and config 1, a kernel summary of config 1, and
# the parity tests of the tail on the new base
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/tests_r05j.log 2>&1 || { tail -20 gpurun_out/tests_r05j.log; exit 1; }
tail -2 gpurun_out/tests_r05j.log
CONFIGS="config3 config1" timeout -k 10 600 bash tools/ab_multi.sh > gpurun_out/ab_r05j.txt 2>&1 || { cat gpurun_out/ab_r05j.txt; exit 2; }
cat gpurun_out/ab_r05j.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05j_c1 -o run -- python3 bench.py --no-cpu-baseline --config config1 --steps 10 --warmup 3 > gpurun_out/prof_r05j_c1.log 2>&1 || exit 3
python3 tools/prof_summary.py $(python3 -c "import glob; print(glob.glob('gpurun_out/prof_r05j_c1/**/*kernel_stats.csv', recursive=True)[0])") 13 > gpurun_out/prof_r05j_c1.txt 2>&1; head -30 gpurun_out/prof_r05j_c1.txt
