# A/B of the row-block reduce's sort (KMP_BINSORT: 0 radix, 2 bins everywhere, 1 default) on
# config 3 and config 5
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 0 2; do
  KMP_BINSORT=$m timeout -k 10 120 python3 bench.py --no-cpu-baseline > gpurun_out/ab_c3_$m.json 2>/dev/null
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_c3_$m.json')); print('c3 mode $m', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in d['roofline']['stages'].items()})"
done
for m in 0 2; do
  KMP_BINSORT=$m timeout -k 10 200 python3 bench.py --config config5 --no-cpu-baseline > gpurun_out/ab_c5_$m.json 2>/dev/null
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_c5_$m.json')); print('c5 mode $m', round(d['ms_per_step']), {k: round(v['ms']) for k,v in d['roofline']['stages'].items()})"
done
