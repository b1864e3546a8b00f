# kernel traces: a G = 8 rank of the sharded split, and the one-GPU config-3 step
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=r05r MODE=sharded timeout -k 10 600 bash tools/prof_split.sh config3 8 > gpurun_out/r05r_split.log 2>&1 || { tail -5 gpurun_out/r05r_split.log; exit 1; }
cat gpurun_out/prof_r05r_g8.txt | head -20
bash tools/profile.sh kernels r05c3b > gpurun_out/r05r_k3.log 2>&1 || { tail -5 gpurun_out/r05r_k3.log; exit 2; }
head -12 gpurun_out/prof_r05c3b.txt
