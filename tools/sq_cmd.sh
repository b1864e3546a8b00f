# Two SQ counter passes (8 counters each) over the kernels matching REGEX of any python command,
# summarised per wave (tools/sq_summary.py) -> gpurun_out/sq_TAG.txt
#   bash tools/sq_cmd.sh TAG REGEX python3 script.py args...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
tag=$1; regex=$2; shift 2
rm -rf gpurun_out/sq1_$tag gpurun_out/sq2_$tag
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "$regex" --output-format csv \
  -d gpurun_out/sq1_$tag -o run -- "$@" > gpurun_out/sq1_$tag.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY --kernel-include-regex "$regex" --output-format csv \
  -d gpurun_out/sq2_$tag -o run -- "$@" > gpurun_out/sq2_$tag.log 2>&1
python3 tools/sq_summary.py gpurun_out/sq1_$tag gpurun_out/sq2_$tag > gpurun_out/sq_$tag.txt
cat gpurun_out/sq_$tag.txt
