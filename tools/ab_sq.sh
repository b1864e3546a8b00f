# SQ counters per wave of the kernels matching $REGEX (default bucket_small) for the in-tree library
# and every tools/ab/<name>/libkmerpair.so variant (one rocprofv3 --pmc pass each) -> gpurun_out/absq_*.txt
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R
for v in base $(ls tools/ab 2>/dev/null); do
  if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$R/tools/ab/$v/libkmerpair.so; fi
  rm -rf gpurun_out/absq_$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_LDS SQ_INSTS_VMEM --kernel-include-regex "${REGEX:-bucket_small}" --output-format csv \
    -d gpurun_out/absq_$v -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/absq_$v.log 2>&1
  python3 tools/sq_summary.py gpurun_out/absq_$v > gpurun_out/absq_$v.txt
  echo "== $v"; cat gpurun_out/absq_$v.txt
done
