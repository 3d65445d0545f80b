# Cache-policy A/B at HEAD (measurement builds): non-temporal map stores,
# non-temporal side loads, stack-load aux bits 0 / 2 (default, nt) / 3 / 18.  -> gpurun_out/r3cpol
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3cpol
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
}
for rep in 1 2; do
  run def_$rep X=1
  for v in ntmaps ntside aux0 aux3 aux18; do run ${v}_$rep SLGPU_LIB=build/libslgpu_$v.so; done
done
python3 - <<'PY'
import json, glob
O = 'gpurun_out/r3cpol'
for f in sorted(glob.glob(f'{O}/*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['path']['kernel_avg_ms']
    print(f.split('/')[-1][:-5].ljust(10), 'us/step %.2f' % (1e3 * d['ms_per_step']), 'frac %.3f' % d['roofline']['frac'],
          'kdec_frac %.3f' % d['roofline']['dominant_kernel']['frac'], ' '.join('%s %.1f' % (n, 1e3 * v) for n, v in k.items()))
PY
