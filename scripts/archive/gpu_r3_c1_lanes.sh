# c1 views in flight with next-stats (2 launches per call): --streams 3/4/6/8, alternating.  -> gpurun_out/r3c1
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3c1
mkdir -p $O
for rep in 1 2; do
  for s in ${LANES:-3 4 6 8}; do
    timeout -k 10 200 python -u bench.py --config c1 --streams $s --no-cpu-baseline --no-secondary > $O/s${s}_$rep.json 2> $O/s${s}_$rep.err || { tail -20 $O/s${s}_$rep.err; exit 1; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/r3c1/*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1][:-5].ljust(8), 'us/step %.2f' % (1e3 * d['ms_per_step']), 'Gpx/s %.1f' % (d['value'] / 1e9), 'frac %.3f' % d['roofline']['frac'])
PY
