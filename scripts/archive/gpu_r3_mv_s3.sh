# Round 3: 2 vs 3 views in flight for c3 / c4 / c5 (exact mode, BASELINE scale).  -> gpurun_out/r3mv3
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3mv3
mkdir -p $O
: > $O/lines.log
for cfg in c3 c4 c5; do
  extra=""
  [ $cfg = c3 ] && extra="--scaling strong"
  for S in 2 3; do
    timeout -k 10 300 python -u bench.py --config $cfg $extra --streams $S --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/$cfg-s$S.json 2> $O/$cfg-s$S.err || { tail -20 $O/$cfg-s$S.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/$cfg-s$S.json').read().strip().splitlines()[-1])
print('$cfg S=$S', 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'])
" | tee -a $O/lines.log
  done
done
