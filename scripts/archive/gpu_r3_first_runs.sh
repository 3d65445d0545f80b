# The driver's condition, repeated: the default bench (driver flags) as the first
# GPU command on a fresh box, then twice more, each a new process.  -> gpurun_out/r3first
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3first
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/run$i.json 2> $O/run$i.err || { tail -20 $O/run$i.err; exit 1; }
done
python3 - <<'PY'
import json
for i in (1, 2, 3):
    d = json.loads(open(f'gpurun_out/r3first/run{i}.json').read().strip().splitlines()[-1])
    t = d['timing']
    print(i, 'ms/step %.4f' % d['ms_per_step'], 'enqueue ms %.3f' % t['host_enqueue_ms'], 'window ms %.3f' % (20 * d['ms_per_step']),
          'event-window median %.1f' % t['step_us']['median'], 'preroll', t['preroll'], 'alt %.4f' % d['alt_xyz_mode']['ms_per_step'])
PY
