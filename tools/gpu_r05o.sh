# A/B: capped scatter at one workgroup per CU (sc1cu), the fast reduce at the compiler's occupancy
# (ftw0), level 2 at 4 waves per SIMD (l2w4); then the per-rank split timing
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 bash tools/ab_multi.sh > gpurun_out/ab_r05o.txt 2>&1 || { cat gpurun_out/ab_r05o.txt; exit 1; }
cat gpurun_out/ab_r05o.txt
timeout -k 10 300 python -u tools/time_dist_rank.py config3 sharded 2 4 8 > gpurun_out/dist_sharded_r05o.txt 2>&1 || exit 2
head -5 gpurun_out/dist_sharded_r05o.txt
