# The round's measurements in one GPU session (each step under its own limit; logs and tables under
# gpurun_out/, copied into profiles/ afterwards): bench lines (configs 3 with the CPU baseline, 1, 2),
# rocprofv3 kernel stats of configs 3 and 1, the FETCH_SIZE / WRITE_SIZE passes of config 3, SQ
# counters of the main kernels, and the per-rank k-mer split (kernel traces and timings at G = 1..8).
#   TAG=r04x [STEPS="bench prof pmc sq split c5"] bash tools/gpu_final.sh
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
TAG=${TAG:-final}
STEPS=${STEPS:-bench prof pmc sq split}
for s in $STEPS; do
  case $s in
  bench)
    timeout -k 10 300 python3 bench.py > gpurun_out/${TAG}_bench_config3.json 2> gpurun_out/${TAG}_bench_config3.err
    timeout -k 10 200 python3 bench.py --config config1 > gpurun_out/${TAG}_bench_config1.json 2> gpurun_out/${TAG}_bench_config1.err
    timeout -k 10 200 python3 bench.py --config config2 > gpurun_out/${TAG}_bench_config2.json 2> gpurun_out/${TAG}_bench_config2.err
    python3 -c "
import json
for c in ('config3', 'config1', 'config2'):
    d = json.load(open('gpurun_out/${TAG}_bench_' + c + '.json')); r = d['roofline']
    print(c, round(d['ms_per_step'], 4), 'frac', round(r['frac'], 3), r['kernel'], {k: round(v['ms'], 4) for k, v in r['stages'].items()})"
    ;;
  prof)
    bash tools/profile.sh kernels ${TAG}_c3
    bash tools/profile.sh kernels ${TAG}_c1 --config config1
    ;;
  pmc)
    bash tools/profile.sh traffic ${TAG}
    ;;
  sq)
    bash tools/profile.sh sq "bucket_small|bp_scatter1p|bp_scatter2g|pt_reduce_fast|pt_scatter_capped" ${TAG}
    ;;
  split)
    TAG=${TAG}_split bash tools/prof_split.sh config3 1 2 4 8
    ;;
  c5)
    # one warm-up pass over the batch first: the first stream allocates its multi-GB pass buffers
    # (~1 s of hipMalloc / hipFree inside the clock otherwise); the CPU baseline is a bounded sample
    timeout -k 10 500 python3 bench.py --config config5 --warmup 1 > gpurun_out/${TAG}_bench_config5.json 2> gpurun_out/${TAG}_bench_config5.err
    tail -c 400 gpurun_out/${TAG}_bench_config5.json
    ;;
  esac
done
