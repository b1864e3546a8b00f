cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in base s64 s128; do
  if [ $v = base ]; then unset KMP_LIB; else export KMP_LIB=$GRAFT_REPO_ROOT/tools/ab/$v/libkmerpair.so; fi
  timeout -k 10 200 python -u tools/time_dist_rank.py config3 sharded 2 8 > gpurun_out/ab_sh_$v.txt 2>&1 || exit 1
  echo $v; sed -n 2,3p gpurun_out/ab_sh_$v.txt
  tail -1 gpurun_out/ab_sh_$v.txt | python3 -c "
import json,sys; d=json.load(sys.stdin)
for g,v in d['ranks'].items():
  r=v['per_rank'][0]; print(g, 'keys', round(r['dev_keys_ms'],4), 'group', round(r['dev_group_ms'],4), 'edges', round(r['dev_edges_ms'],4))"
done
unset KMP_LIB
