# Kernel traces of one rank of the k-mer split (tools/prof_split_rank.py) and per-rank wall times
# (tools/time_dist_rank.py), logs under gpurun_out/.
#   TAG=x [MODE=kmer|sharded] bash tools/prof_split.sh [config3|config1] [G ...]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
TAG=${TAG:-split}
cfg=${1:-config3}; shift || true
GS=${*:-1 8}
for g in $GS; do
  rm -rf gpurun_out/prof_${TAG}_g$g
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_g$g -o run -- \
    python3 tools/prof_split_rank.py $cfg $g 0 30 ${MODE:-kmer} > gpurun_out/prof_${TAG}_g$g.log 2>&1
  python3 tools/prof_summary.py $(find gpurun_out/prof_${TAG}_g$g -name 'run_kernel_stats.csv' | head -1) > gpurun_out/prof_${TAG}_g$g.txt
  head -30 gpurun_out/prof_${TAG}_g$g.txt
done
timeout -k 10 300 python3 tools/time_dist_rank.py $cfg ${MODE:-kmer} $GS > gpurun_out/time_${TAG}.txt 2>&1
head -4 gpurun_out/time_${TAG}.txt
