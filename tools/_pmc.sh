# HBM traffic per stage of the config-3 step: separate FETCH_SIZE and WRITE_SIZE passes (kernel
# trace only), summarised by tools/pmc_traffic.py into gpurun_out/pmc_traffic.json
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1
echo fetch done
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_write.log 2>&1
echo write done
python3 tools/pmc_traffic.py $(find gpurun_out/pmc_fetch -name 'run_counter_collection.csv') $(find gpurun_out/pmc_write -name 'run_counter_collection.csv') gpurun_out/pmc_traffic.json
