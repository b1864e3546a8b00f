# A/B: the step's host waits polling the stream (spin=1, default) against hipStreamSynchronize (spin=0)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in config3 config1 config2; do
  for i in 1 2; do
    for v in 1 0; do
      KMP_SPIN=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --config $cfg --steps 40 > gpurun_out/ab_spin$v.json 2>/dev/null || exit 1
      python3 -c "
import json; d=json.load(open('gpurun_out/ab_spin$v.json')); print('$cfg spin=$v', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in d['roofline']['stages'].items()})"
    done
  done
done
