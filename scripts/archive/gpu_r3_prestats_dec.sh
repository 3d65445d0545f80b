# Pre-stats in k_decode's tail (SLGPU_PRE_DECODE=1) vs k_cloud's (default):
# tests, then same-box A/B at c2 and c1 (alternating, 3 rounds).  -> gpurun_out/r3predec
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3predec
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prestats.py > $O/pytest_prestats.log 2>&1 || { tail -40 $O/pytest_prestats.log; exit 1; }
tail -1 $O/pytest_prestats.log
run() {  # name, config, env...
  local n=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --no-secondary > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
}
for rep in 1 2 3; do
  run c2_cloud_$rep c2 X=1
  run c2_dec_$rep c2 SLGPU_PRE_DECODE=1
  run c2_dec_w512_$rep c2 SLGPU_PRE_DECODE=1 SLGPU_PRE_WGS=512
done
for rep in 1 2; do
  run c1_cloud_$rep c1 X=1
  run c1_dec_$rep c1 SLGPU_PRE_DECODE=1
  run c4_cloud_$rep c4 X=1
  run c4_dec_$rep c4 SLGPU_PRE_DECODE=1
done
python3 - <<'PY'
import json, glob
O = 'gpurun_out/r3predec'
for f in sorted(glob.glob(f'{O}/*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['path']['kernel_avg_ms']
    print(f.split('/')[-1][:-5].ljust(18), 'us/step %.2f' % (1e3 * d['ms_per_step']), 'frac %.3f' % d['roofline']['frac'],
          'med %.1f' % d['timing']['step_us']['median'], ' '.join('%s %.1f' % (n, 1e3 * v) for n, v in k.items()))
PY
