# A/B repeated: level 2 tile-major (base) against bin-major (binmaj), config 3, 40 steps, three rounds
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2 3; do
  for v in base binmaj; do
    if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/$v/libkmerpair.so; fi
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); print('config3', '$v'.ljust(6), round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in d['roofline']['stages'].items()})"
  done
done
