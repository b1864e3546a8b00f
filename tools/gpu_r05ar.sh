# final check of the committed tree after the reverted experiment: the GPU suite, smoke(), the default bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r05ar_tests.log 2>&1 || { tail -20 gpurun_out/r05ar_tests.log; exit 1; }
tail -1 gpurun_out/r05ar_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05ar_smoke.log 2>&1 || { tail -5 gpurun_out/r05ar_smoke.log; exit 2; }
tail -1 gpurun_out/r05ar_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r05ar_bench.json 2> gpurun_out/r05ar_bench.err || exit 3
python3 -c "
import json; d=json.load(open('gpurun_out/r05ar_bench.json')); print(d['metric'], round(d['ms_per_step'],4), d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
