# cost of the stage events in the timed step: config 3 and 1 with (timing=1) and without (timing=0) them
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in config3 config1; do
  for i in 1 2 3; do
    for v in 1 0; do
      if [ $v = 0 ]; then export BENCH_NO_STAGE_TIMING=1; else unset BENCH_NO_STAGE_TIMING; fi
      timeout -k 10 120 python3 bench.py --no-cpu-baseline --config $cfg --steps 40 > gpurun_out/ab_tm$v.json 2>/dev/null || exit 1
      python3 -c "
import json; d=json.load(open('gpurun_out/ab_tm$v.json')); print('$cfg timing=$v', round(d['ms_per_step'],4))"
    done
  done
done
