# A/B: segment sorts before the read-back (default) vs after it (KMP_PRESORT=0), config 1, alternating
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 1 0; do
    KMP_PRESORT=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --config config1 --steps 40 > gpurun_out/ab_pre$v.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_pre$v.json')); print('presort=$v', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in d['roofline']['stages'].items()})"
  done
done
