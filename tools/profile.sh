# Profiling recipes for the GPU box (each step under its own time limit; logs under gpurun_out/).
#   bash tools/profile.sh kernels TAG [bench args]   kernel trace + stats of bench.py -> gpurun_out/prof_TAG
#   bash tools/profile.sh traffic TAG                FETCH_SIZE and WRITE_SIZE passes of the config-3 bench
#                                                    -> gpurun_out/pmc_traffic_TAG.json (tools/pmc_traffic.py)
#   bash tools/profile.sh traffic5 TAG               the same over one config-5 step (reduce + expansion kernels)
#                                                    -> gpurun_out/pmc_config5_TAG.json (tools/pmc_config5.py)
#   bash tools/profile.sh sq REGEX TAG               two SQ counter passes (8 counters each) over the kernels
#                                                    matching REGEX -> gpurun_out/sq_TAG.txt
#   bash tools/profile.sh sq5 REGEX TAG              the same over one cold config-5 step
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
mode=$1; shift
case $mode in
kernels)
  tag=$1; shift
  rm -rf gpurun_out/prof_$tag
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
    python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err
  python3 tools/prof_summary.py $(find gpurun_out/prof_$tag -name 'run_kernel_stats.csv' | head -1) > gpurun_out/prof_$tag.txt
  head -24 gpurun_out/prof_$tag.txt
  ;;
traffic)
  tag=$1
  rm -rf gpurun_out/pmc_fetch_$tag gpurun_out/pmc_write_$tag
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$tag -o run -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_fetch_$tag.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$tag -o run -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_write_$tag.log 2>&1
  python3 tools/pmc_traffic.py $(find gpurun_out/pmc_fetch_$tag -name 'run_counter_collection.csv') \
    $(find gpurun_out/pmc_write_$tag -name 'run_counter_collection.csv') gpurun_out/pmc_traffic_$tag.json
  ;;
traffic5)
  # config 5: the fused reduce's and the expansion's kernels only (one step; each pass its own run)
  tag=$1
  # (the warm step: one warm-up stream, then the marker kernel the table starts after)
  re="pt_hist|pt_tscan|pt_scatter_kernel|pt_split|pt_window_count|pt_reduce_count|pt_reduce_write|heavy_flat|heavy_rows|bucket_small|bucket_large|edge_digest|spin_kernel"
  rm -rf gpurun_out/pmc5_fetch_$tag gpurun_out/pmc5_write_$tag
  timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$re" --output-format csv -d gpurun_out/pmc5_fetch_$tag -o run -- \
    python3 bench.py --config config5 --no-cpu-baseline --warmup 1 > gpurun_out/pmc5_fetch_$tag.log 2>&1
  timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$re" --output-format csv -d gpurun_out/pmc5_write_$tag -o run -- \
    python3 bench.py --config config5 --no-cpu-baseline --warmup 1 > gpurun_out/pmc5_write_$tag.log 2>&1
  python3 tools/pmc_config5.py $(find gpurun_out/pmc5_fetch_$tag -name 'run_counter_collection.csv') \
    $(find gpurun_out/pmc5_write_$tag -name 'run_counter_collection.csv') gpurun_out/pmc_config5_$tag.json
  ;;
sq|sq5)
  regex=$1; tag=$2
  cmd="python3 bench.py --no-cpu-baseline --steps 3 --warmup 1"
  [ $mode = sq5 ] && cmd="python3 bench.py --config config5 --no-cpu-baseline --warmup 0" 
  rm -rf gpurun_out/sq1_$tag gpurun_out/sq2_$tag
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "$regex" --output-format csv \
    -d gpurun_out/sq1_$tag -o run -- $cmd > gpurun_out/sq1_$tag.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY --kernel-include-regex "$regex" --output-format csv \
    -d gpurun_out/sq2_$tag -o run -- $cmd > gpurun_out/sq2_$tag.log 2>&1
  python3 tools/sq_summary.py gpurun_out/sq1_$tag gpurun_out/sq2_$tag > gpurun_out/sq_$tag.txt
  cat gpurun_out/sq_$tag.txt
  ;;
esac
