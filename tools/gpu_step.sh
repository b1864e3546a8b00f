# Run GPU steps in order, each under its own limit; a test failure (exit 1) does not stop the next
# step, a time limit, abort or fault (124, 137, 134, 139, ...) does.  Logs under gpurun_out/.
#   bash tools/gpu_step.sh LIMIT_S LOG -- cmd args   (one step; exit code passed through)
lim=$1; log=$2; shift 3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
rc=$?
echo "step $log rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 99; fi
exit 0
