# k_decode at 4 waves per SIMD (measurement builds, scripts/build_variants.sh):
# pl3w4 = packed 12-B plane table (38.4 KB of LDS tables) + launch bounds 4 +
# grid cap 4 per CU; pl3w3 = the packed table alone.  Parity on the variant,
# then same-box bench A/Bs (alternating).  -> gpurun_out/r3pl3
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3pl3
mkdir -p $O
SLGPU_LIB=build/libslgpu_pl3w4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_prestats.py > $O/pytest_pl3w4.log 2>&1 || { tail -40 $O/pytest_pl3w4.log; exit 1; }
tail -1 $O/pytest_pl3w4.log
run() {  # name, config, env...
  local n=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --no-secondary > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
}
for rep in 1 2 3; do
  run c2_def_$rep c2 X=1
  run c2_pl3w4_$rep c2 SLGPU_LIB=build/libslgpu_pl3w4.so
  run c2_pl3w3_$rep c2 SLGPU_LIB=build/libslgpu_pl3w3.so
done
for rep in 1 2; do
  run c4_def_$rep c4 X=1
  run c4_pl3w4_$rep c4 SLGPU_LIB=build/libslgpu_pl3w4.so
  run c3_def_$rep c3 X=1
  run c3_pl3w4_$rep c3 SLGPU_LIB=build/libslgpu_pl3w4.so
done
python3 - <<'PY'
import json, glob
O = 'gpurun_out/r3pl3'
for f in sorted(glob.glob(f'{O}/*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['path']['kernel_avg_ms']
    print(f.split('/')[-1][:-5].ljust(14), 'us/step %.2f' % (1e3 * d['ms_per_step']), 'frac %.3f' % d['roofline']['frac'],
          'kdec_frac %.3f' % d['roofline']['dominant_kernel']['frac'], ' '.join('%s %.1f' % (n, 1e3 * v) for n, v in k.items()))
PY
