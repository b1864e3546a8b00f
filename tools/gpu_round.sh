# One GPU session, as a list of steps (each under its own time limit; logs and tables under
# gpurun_out/, copied into profiles/ by hand afterwards).  The one script for every GPU call:
#   TAG=r06x STEPS="tests bench ab prof pmc sq sq5 split c5 c5rank c5ev" [options] bash tools/gpu_round.sh
# steps:
#   tests  pytest -m gpu (PYTEST_K / PYTEST_FILES select; tools/gpu_tests.sh)
#   bench  bench lines of CONFIGS (default "config3 config1 config2"); config 3 with the CPU baseline
#   ab     A/B of the in-tree library against tools/ab/<name>/libkmerpair.so (tools/ab_multi.sh),
#          over AB_CONFIGS (default config3), AB_ROUNDS alternations (default 2)
#   prof   rocprofv3 kernel stats of the config-3 and config-1 benches (tools/profile.sh kernels)
#   pmc    FETCH_SIZE / WRITE_SIZE passes of the config-3 bench (tools/profile.sh traffic)
#   sq     SQ counters of the kernels matching SQ_REGEX (default: the step's five main kernels)
#   sq5    the same over one cold config-5 step (SQ5_REGEX: the reduce's and expansion's kernels)
#   split  the k-mer split's per-rank kernel traces and wall times at SPLIT_G (default "1 8"), MODE
#          kmer | sharded (tools/prof_split.sh)
#   c5     the config-5 bench line (one warm-up stream; its CPU baseline sample)
#   c5rank config 5's per-rank share at G ranks: one rank's rows streamed alone (bench --rank-of R/G
#          for RANKS, default "0/8 7/8 0/100000": the largest and last of an 8-rank split, and a rank
#          of ~10 rows, i.e. the replicated front alone)
#   c5ev   config-5 evidence of one command: its PMC table (tools/profile.sh traffic5), bench line
#          and the kernel summary of the warm step (tools/trace_after_marker.py)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
TAG=${TAG:-round}
STEPS=${STEPS:-tests bench}
summary() {  # bench line -> one printed line
  python3 -c "
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
print(sys.argv[2], round(d['ms_per_step'], 4), 'frac', round(r['frac'], 3), {k: round(v['ms'], 4) for k, v in r.get('stages', {}).items()})" "$1" "$2"
}
for s in $STEPS; do
  case $s in
  tests)
    TAG=$TAG bash tools/gpu_tests.sh
    ;;
  bench)
    for c in ${CONFIGS:-config3 config1 config2}; do
      cb=--no-cpu-baseline
      [ $c = config3 ] && cb=
      timeout -k 10 300 python3 bench.py $cb --config $c > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err
      summary gpurun_out/${TAG}_bench_$c.json $c
    done
    ;;
  ab)
    CONFIGS=${AB_CONFIGS:-config3} ROUNDS=${AB_ROUNDS:-2} timeout -k 10 900 bash tools/ab_multi.sh
    ;;
  prof)
    bash tools/profile.sh kernels ${TAG}_c3
    bash tools/profile.sh kernels ${TAG}_c1 --config config1
    ;;
  pmc)
    bash tools/profile.sh traffic ${TAG}
    python3 -c "
import json; d = json.load(open('gpurun_out/pmc_traffic_${TAG}.json'))
print({k: round(v['bytes'] / 1e6, 1) for k, v in d['stages'].items()}, 'total MB', round(sum(v['bytes'] for v in d['stages'].values()) / 1e6, 1))"
    ;;
  sq)
    bash tools/profile.sh sq "${SQ_REGEX:-bucket_small|bp_scatter1p|bp_scatter2g|pt_reduce_fast|pt_scatter_capped}" ${TAG}
    ;;
  sq5)
    bash tools/profile.sh sq5 "${SQ5_REGEX:-pt_reduce_count|pt_split|heavy_rows|pt_reduce_write}" ${TAG}_c5
    ;;
  split)
    TAG=${TAG}_split bash tools/prof_split.sh config3 ${SPLIT_G:-1 8}
    ;;
  c5)
    timeout -k 10 500 python3 bench.py --config config5 --warmup 1 > gpurun_out/${TAG}_bench_config5.json 2> gpurun_out/${TAG}_bench_config5.err
    summary gpurun_out/${TAG}_bench_config5.json config5
    ;;
  c5rank)
    for rg in ${RANKS:-0/8 7/8 0/100000}; do
      t=$(echo $rg | tr / _)
      timeout -k 10 300 python3 bench.py --config config5 --warmup 1 --no-cpu-baseline --rank-of $rg > gpurun_out/${TAG}_c5rank_$t.json 2> gpurun_out/${TAG}_c5rank_$t.err
      python3 -c "
import json, sys; d = json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'], 1), d.get('emulated_rank'))" gpurun_out/${TAG}_c5rank_$t.json $rg
    done
    ;;
  c5ev)
    bash tools/profile.sh traffic5 ${TAG} > gpurun_out/${TAG}_traffic5.log 2>&1
    timeout -k 10 500 python3 bench.py --config config5 --warmup 1 > gpurun_out/${TAG}_bench_config5.json 2> gpurun_out/${TAG}_bench_config5.err
    summary gpurun_out/${TAG}_bench_config5.json config5
    rm -rf gpurun_out/prof_${TAG}_c5
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_c5 -o run -- \
      python3 bench.py --config config5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}_c5.json 2> gpurun_out/prof_${TAG}_c5.err
    python3 tools/trace_after_marker.py $(find gpurun_out/prof_${TAG}_c5 -name 'run_kernel_trace.csv') > gpurun_out/prof_${TAG}_c5.txt
    head -16 gpurun_out/prof_${TAG}_c5.txt
    rm -f $(find gpurun_out/prof_${TAG}_c5 -name 'run_kernel_trace.csv')
    ;;
  *)
    echo "unknown step $s"; exit 2
    ;;
  esac
done
