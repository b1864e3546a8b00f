# SQ counters of config 1's main kernels (two passes) and its FETCH/WRITE per kernel (two passes)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
re="bucket_small|bucket_large|pt_reduce_kernel|pt_scatter_kernel|pt_rowhist|heavy_seg|heavy_expand|pt_emit"
rm -rf gpurun_out/sq1_c1 gpurun_out/sq2_c1 gpurun_out/fe_c1 gpurun_out/wr_c1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "$re" --output-format csv \
  -d gpurun_out/sq1_c1 -o run -- python3 bench.py --no-cpu-baseline --config config1 --steps 3 --warmup 1 > gpurun_out/sq1_c1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY --kernel-include-regex "$re" --output-format csv \
  -d gpurun_out/sq2_c1 -o run -- python3 bench.py --no-cpu-baseline --config config1 --steps 3 --warmup 1 > gpurun_out/sq2_c1.log 2>&1 || exit 2
python3 tools/sq_summary.py gpurun_out/sq1_c1 gpurun_out/sq2_c1 > gpurun_out/sq_c1.txt
cat gpurun_out/sq_c1.txt | cut -c1-200
