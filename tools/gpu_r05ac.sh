# A/B: level 2 tile-major workgroup order (tmaj) against bin-major (base): bench on configs 3 and 1,
# then FETCH_SIZE of bp_scatter2g for each
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
CONFIGS="config3 config1" timeout -k 10 600 bash tools/ab_multi.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base tmaj; do
  if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/$v/libkmerpair.so; fi
  rm -rf gpurun_out/pmc_l2_$v
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "bp_scatter2g" --output-format csv -d gpurun_out/pmc_l2_$v -o run -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_l2_$v.log 2>&1 || exit 2
  python3 -c "
import csv, glob
f = glob.glob('gpurun_out/pmc_l2_$v/**/run_counter_collection.csv', recursive=True)[0]
v = [float(r['Counter_Value']) for r in csv.DictReader(open(f)) if r['Counter_Name'] == 'FETCH_SIZE']
print('$v FETCH_SIZE per launch (KB):', [round(x) for x in v[-3:]])"
done
