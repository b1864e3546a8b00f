# the split step's front as a graph: full GPU suite, config 1 A/B against launches call by call (KMP_FRONT_GRAPH=0), config 5 once
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r05aq_tests.log 2>&1 || { tail -20 gpurun_out/r05aq_tests.log; exit 1; }
tail -1 gpurun_out/r05aq_tests.log
for i in 1 2 3; do
  for v in 1 0; do
    KMP_FRONT_GRAPH=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --config config1 --steps 40 > gpurun_out/ab_fg$v.json 2>/dev/null || exit 2
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_fg$v.json')); print('config1 front_graph=$v', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in d['roofline']['stages'].items()})"
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --config config5 --warmup 1 > gpurun_out/r05aq_c5.json 2> gpurun_out/r05aq_c5.err || exit 3
python3 -c "
import json; d=json.load(open('gpurun_out/r05aq_c5.json')); print('config5', round(d['ms_per_step'],1))"
