# heavy segment sizes at configs 1 and 3 (KMP_TRACE diagnostics)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
KMP_TRACE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --config config1 --steps 1 --warmup 1 > gpurun_out/r05v_c1.json 2> gpurun_out/r05v_c1.err || exit 1
grep "segs" gpurun_out/r05v_c1.err | sort | uniq -c | head -40
KMP_TRACE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/r05v_c3.json 2> gpurun_out/r05v_c3.err || exit 2
grep -c "segs" gpurun_out/r05v_c3.err; grep "segs" gpurun_out/r05v_c3.err | sort | uniq -c | head -20; true
