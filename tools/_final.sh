# round-end measurements: GPU tests, bench lines (configs 3, 1, 2; config 3 with its CPU
# baseline), kernel-trace stats of configs 3 and 1, PMC traffic, per-rank multi-GPU emulation
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/_gpu_tests.sh
timeout -k 10 400 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
echo c3; cat gpurun_out/bench_c3.json
timeout -k 10 300 python bench.py --config config1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err
timeout -k 10 300 python bench.py --config config2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
echo benches done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_c3 gpurun_out/prof_c1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_c3.json 2> gpurun_out/prof_c3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1 -o run -- python3 bench.py --config config1 --no-cpu-baseline > gpurun_out/prof_c1.json 2> gpurun_out/prof_c1.err
python tools/prof_summary.py $(find gpurun_out/prof_c3 -name 'run_kernel_stats.csv' | head -1) 24 > gpurun_out/summary_c3.txt
python tools/prof_summary.py $(find gpurun_out/prof_c1 -name 'run_kernel_stats.csv' | head -1) 25 > gpurun_out/summary_c1.txt
echo profiles done
bash tools/_pmc.sh
timeout -k 10 300 python tools/time_dist_rank.py config3 kmer 1 2 4 8 > gpurun_out/dist_kmer.txt 2>&1
timeout -k 10 300 python tools/time_dist_rank.py config3 rows 1 2 4 8 > gpurun_out/dist_rows.txt 2>&1
echo all done
