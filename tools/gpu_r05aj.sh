# heavy plan and expansion sized by the segment bound: full GPU suite, config-1/3 bench, config-1 kernels
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r05aj_tests.log 2>&1 || { tail -20 gpurun_out/r05aj_tests.log; exit 1; }
tail -2 gpurun_out/r05aj_tests.log
for c in config1 config3 config1 config3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/r05aj_$c.json 2> gpurun_out/r05aj_$c.err || exit 2
  python3 -c "
import json; d=json.load(open('gpurun_out/r05aj_$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],4), {k: round(v['ms'],4) for k,v in r['stages'].items()})"
done
bash tools/profile.sh kernels r05aj1 --config config1 > gpurun_out/r05aj_k1.log 2>&1 || exit 3
head -24 gpurun_out/prof_r05aj1.txt
