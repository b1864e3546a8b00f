set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1
echo fetch done
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_write.log 2>&1
echo write done
