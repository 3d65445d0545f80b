# Multi-view configs' views in flight with next-stats: c3 (strong, 36 views) and c5 (45 views) at --streams 1/2/3.  -> gpurun_out/r3mv
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3mv
mkdir -p $O
for rep in 1 2; do
  for s in 1 2 3; do
    timeout -k 10 300 python -u bench.py --config c3 --scaling strong --streams $s --no-cpu-baseline --no-secondary > $O/c3_s${s}_$rep.json 2> $O/c3_s${s}_$rep.err || { tail -20 $O/c3_s${s}_$rep.err; exit 1; }
  done
done
for s in 1 2 3; do
  timeout -k 10 300 python -u bench.py --config c5 --streams $s --no-cpu-baseline --no-secondary > $O/c5_s${s}.json 2> $O/c5_s${s}.err || { tail -20 $O/c5_s${s}.err; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/r3mv/*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1][:-5].ljust(10), 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value'] / 1e9), 'frac %.3f' % d['roofline']['frac'])
PY
