# per-rank row-split timing (config3) + SQ counter passes of the bucket kernel
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/time_dist_rank.py config3 > gpurun_out/dist_rank_c3.txt 2>&1
tail -5 gpurun_out/dist_rank_c3.txt | cut -c1-300
bash tools/_pmc_bucket.sh bucket_small
