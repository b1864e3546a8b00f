# A/B: mean keys per bucket target (layout bbits): 1024 (base), 512, 2048; configs 3 and 1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
CONFIGS="config3 config1" timeout -k 10 800 bash tools/ab_multi.sh || exit 1
