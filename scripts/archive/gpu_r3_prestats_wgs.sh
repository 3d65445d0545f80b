# Pre-stats grid size A/B at c2 (same box, alternating, 3 rounds).  -> gpurun_out/r3prewgs
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3prewgs
mkdir -p $O
run() {  # name, config, env...
  local n=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --no-secondary > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
}
for rep in 1 2 3; do
  run c2_w512_$rep c2 X=1
  run c2_w1024_$rep c2 SLGPU_PRE_WGS=1024
  run c2_w1536_$rep c2 SLGPU_PRE_WGS=1536
  run c2_w2048_$rep c2 SLGPU_PRE_WGS=2048
  run c2_off_$rep c2 SLGPU_PRESTATS=0
done
python3 - <<'PY'
import json, glob
O = 'gpurun_out/r3prewgs'
for f in sorted(glob.glob(f'{O}/*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['path']['kernel_avg_ms']
    print(f.split('/')[-1][:-5].ljust(18), 'us/step %.2f' % (1e3 * d['ms_per_step']), 'frac %.3f' % d['roofline']['frac'],
          'med %.1f' % d['timing']['step_us']['median'], ' '.join('%s %.1f' % (n, 1e3 * v) for n, v in k.items()))
PY
