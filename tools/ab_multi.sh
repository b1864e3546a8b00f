# A/B of the bench over library variants: base (in-tree) and tools/ab/<name>/libkmerpair.so,
# alternating, ROUNDS times (default 2); CONFIGS (default "config3") picks the bench configs, AB_ARGS
# adds bench arguments (config 5: --warmup 1)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in ${CONFIGS:-config3}; do
  for i in $(seq ${ROUNDS:-2}); do
    for v in base $(ls tools/ab 2>/dev/null); do
      if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/$v/libkmerpair.so; fi
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --config $cfg ${AB_ARGS:-} > gpurun_out/ab_$v.json 2>/dev/null
      python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$cfg', '$v'.ljust(6), round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in d['roofline']['stages'].items()})"
    done
  done
done
