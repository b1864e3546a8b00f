set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base old dpp base; do
  if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/$v/libkmerpair.so; fi
  timeout -k 10 200 python3 bench.py --config config5 --no-cpu-baseline > gpurun_out/c5_$v.json 2>/dev/null
  python3 -c "
import json; d=json.load(open('gpurun_out/c5_$v.json')); r=d['roofline']; print('$v', round(d['ms_per_step'],1), d['digest'], {k: round(v['ms'],1) for k,v in r['stages'].items()})"
done
