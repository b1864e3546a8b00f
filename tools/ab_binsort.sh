# A/B of the row-block reduce's sort on config 3 and config 5: builds the library with
# KMP_BINSORT_MODE=0 (radix everywhere) and =2 (bins everywhere) into tools/ab/ (run on the CPU
# side first: bash tools/ab_binsort.sh build), then the A/B on the GPU box (bash tools/ab_binsort.sh)
set -e
if [ "$1" = build ]; then
  bash "$(dirname "$0")/ab_build.sh" bs0 -DKMP_BINSORT_MODE=0
  bash "$(dirname "$0")/ab_build.sh" bs2 -DKMP_BINSORT_MODE=2
  exit 0
fi
cd $GRAFT_REPO_ROOT
CONFIGS="config3 config5" bash tools/ab_multi.sh
