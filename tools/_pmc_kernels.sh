# one SQ counter pass (8 counters, PMC_COUNTERS overrides) over the config-3 bench for the kernels matching $1
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -rf gpurun_out/pmck
timeout -s KILL 120 rocprofv3 --pmc ${PMC_COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES} --kernel-include-regex "$1" --output-format csv -d gpurun_out/pmck -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmck.log 2>&1
python3 - <<'PY'
import csv, glob, collections, sys
sys.path.insert(0, 'tools')
from prof_summary import short
for f in glob.glob('gpurun_out/pmck/**/run_counter_collection.csv', recursive=True):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(short(r['Kernel_Name'])[-48:], r['Counter_Name'])].append(float(r['Counter_Value']))
    names = sorted({k[0] for k in agg})
    for n in names:
        w = sum(agg[(n, 'SQ_WAVES')]) / len(agg[(n, 'SQ_WAVES')])
        print(n, {c: round(sum(v) / len(v) / max(w, 1), 1) for (m, c), v in agg.items() if m == n}, 'waves', w)
PY
