# k_cloud variants with pre-stats (measurement builds): launch bounds 4 waves (cw4), 1 point per lane per pass on the verified route (vp1).  -> gpurun_out/r3cv
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3cv
mkdir -p $O
run() { local n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for rep in 1 2 3; do
  run def_$rep X=1
  run cw4_$rep SLGPU_LIB=build/libslgpu_cw4.so
  run vp1_$rep SLGPU_LIB=build/libslgpu_vp1.so
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/r3cv/*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['path']['kernel_avg_ms']
    print(f.split('/')[-1][:-5].ljust(8), 'us/step %.2f' % (1e3 * d['ms_per_step']), 'frac %.3f' % d['roofline']['frac'], ' '.join('%s %.1f' % (n, 1e3 * v) for n, v in k.items()))
PY
