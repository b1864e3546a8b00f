# One GPU session: the GPU tests (+ bench line), the A/B of tools/ab/* variants, and the k-mer
# split's per-rank kernel traces.  Each step under its own limit; logs under gpurun_out/.
#   TAG=x [SKIP_TESTS=1] [SPLIT_G="1 8"] bash tools/gpu_round.sh
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-round}
if [ -z "$SKIP_TESTS" ]; then
  TAG=$TAG BENCH=1 bash tools/gpu_tests.sh
fi
if [ -d tools/ab ] && [ -n "$(ls tools/ab)" ]; then
  bash tools/ab_multi.sh
fi
if [ -n "$SPLIT_G" ]; then
  TAG=$TAG bash tools/prof_split.sh config3 $SPLIT_G
fi
