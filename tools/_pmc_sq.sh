# one SQ counter pass over a short bench (wave-cycle breakdown per kernel) -> gpurun_out/pmc_sq
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmc_sq.log 2>&1
echo sq done
