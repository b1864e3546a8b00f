# bench stage times for each build_variants/libkmerpair_*.so (argument: variant names)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "$@"; do
  KMP_LIB=$PWD/build_variants/libkmerpair_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']
print('$v', 'ms/step %.3f' % d['ms_per_step'], 'edges', d['config']['edges'], r['layout'], {k: round(v['ms'],3) for k,v in r['stages'].items()})"
done
