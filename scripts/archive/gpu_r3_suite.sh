# Full GPU suite, then the c1 / c3 / c4 / c5 config lines at HEAD defaults.  -> gpurun_out/r3suite
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3suite
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for cfg in c1 c3 c4 c5; do
  extra=""
  [ $cfg = c3 ] && extra="--scaling strong"
  timeout -k 10 600 python -u bench.py --config $cfg $extra --no-cpu-baseline --no-secondary > $O/$cfg.json 2> $O/$cfg.err || { tail -20 $O/$cfg.err; exit 1; }
  timeout -k 10 600 python -u bench.py --config $cfg $extra --no-cpu-baseline --no-secondary --no-next-stats > $O/${cfg}_off.json 2> $O/${cfg}_off.err || { tail -20 $O/${cfg}_off.err; exit 1; }
done
python3 - <<'PY'
import json, glob
O = 'gpurun_out/r3suite'
for f in sorted(glob.glob(f'{O}/c*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1][:-5].ljust(8), 'ms %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value'] / 1e9), 'frac %.3f' % d['roofline']['frac'])
PY
