# FETCH_SIZE / WRITE_SIZE calibration (tools/pmc_calib.hip): timing run, then one PMC pass per
# counter, summarised into gpurun_out/pmc_calib.json by tools/pmc_calib.py
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 tools/pmc_calib 1024 2 > gpurun_out/pmc_calib_time.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/calib_fetch gpurun_out/calib_write
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_fetch -o run -- tools/pmc_calib 1024 2 > /dev/null
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib_write -o run -- tools/pmc_calib 1024 2 > /dev/null
python3 tools/pmc_calib.py $(find gpurun_out/calib_fetch -name 'run_counter_collection.csv') $(find gpurun_out/calib_write -name 'run_counter_collection.csv') $((1024 * 1048576)) gpurun_out/pmc_calib.json
