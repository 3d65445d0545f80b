# Pre-stats placement A/B at c2 / c1 (same box, alternating): after k_cloud's
# workgroups (default) or spread among them (SLGPU_PRE_MIX=1), and the
# pre-stats grid size (SLGPU_PRE_WGS).  -> gpurun_out/r3preab
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3preab
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prestats.py > $O/pytest_prestats.log 2>&1 || { tail -40 $O/pytest_prestats.log; exit 1; }
tail -1 $O/pytest_prestats.log
run() {  # name, config, env...
  local n=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --no-secondary > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
}
for rep in 1 2; do
  run c2_def_$rep c2 X=1
  run c2_mix_$rep c2 SLGPU_PRE_MIX=1
  run c2_w256_$rep c2 SLGPU_PRE_WGS=256
  run c2_w128_$rep c2 SLGPU_PRE_WGS=128
  run c2_mix_w256_$rep c2 SLGPU_PRE_MIX=1 SLGPU_PRE_WGS=256
  run c2_w1024_$rep c2 SLGPU_PRE_WGS=1024
done
for rep in 1 2; do
  run c1_def_$rep c1 X=1
  run c1_mix_$rep c1 SLGPU_PRE_MIX=1
  run c1_w128_$rep c1 SLGPU_PRE_WGS=128
done
python3 - <<'PY'
import json, glob
O = 'gpurun_out/r3preab'
for f in sorted(glob.glob(f'{O}/*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['path']['kernel_avg_ms']
    print(f.split('/')[-1][:-5].ljust(18), 'us/step %.2f' % (1e3 * d['ms_per_step']), 'frac %.3f' % d['roofline']['frac'],
          'med %.1f' % d['timing']['step_us']['median'], ' '.join('%s %.1f' % (n, 1e3 * v) for n, v in k.items()))
PY
