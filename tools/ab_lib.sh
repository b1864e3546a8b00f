# A/B of the config-3 bench: the in-tree library vs tools/ab/libkmerpair.so (KMP_LIB), alternating
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for v in base ab; do
    if [ $v = ab ]; then export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/libkmerpair.so; else unset KMP_LIB; fi
    timeout -k 10 120 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/ab_$v.json 2>/dev/null
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in d['roofline']['stages'].items()})"
  done
done
