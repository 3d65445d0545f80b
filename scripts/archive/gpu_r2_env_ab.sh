# Same-box A/B of an environment switch on bench.py config lines: arguments are
# "label|ENV=VAL ..." pairs; configs from AB_CONFIGS (default "c3 c4 c5"); each
# variant runs twice, interleaved.  -> gpurun_out/eab
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/eab
mkdir -p $O
for rep in 1 2; do
  for cfg in ${AB_CONFIGS:-c3 c4 c5}; do
    for spec in "$@"; do
      IFS='|' read -r label envs <<< "$spec"
      env $envs timeout -k 10 200 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > $O/b.json 2>/dev/null || exit 1
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('$label'.ljust(8), '$cfg'.ljust(4), 'us/step %.1f'%(d['ms_per_step']*1e3), 'path %.3f'%d['roofline']['frac'], 'kdec %.3f'%d['roofline']['dominant_kernel']['frac'], {k: round(v*1e3,1) for k,v in d['path']['rerun_ms_last_group'].items() if isinstance(v,float)})"
    done
  done
done
