# Round 3: views in flight for the multi-view configs in the exact mode
# (c3 strong 36 views, c4 45 views): --streams 1 vs 2, interleaved.  -> gpurun_out/r3mvs
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3mvs
mkdir -p $O
: > $O/lines.log
for cfg in c3 c4; do
  extra=""
  [ $cfg = c3 ] && extra="--scaling strong"
  for rep in 1 2; do
    for S in 1 2; do
      timeout -k 10 300 python -u bench.py --config $cfg $extra --streams $S --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/$cfg-s$S-$rep.json 2> $O/$cfg-s$S-$rep.err || { tail -20 $O/$cfg-s$S-$rep.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('$O/$cfg-s$S-$rep.json').read().strip().splitlines()[-1])
print('$cfg S=$S', 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'])
" | tee -a $O/lines.log
    done
  done
done
