# Same-box A/B of the exact (f64-arithmetic) k_cloud: bench lines of config 5
# (pose) and config 2 with --xyz exact, per library, twice interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/xab
mkdir -p $O
for rep in 1 2; do
  for spec in "$@"; do
    IFS='|' read -r label lib <<< "$spec"
    [ "$lib" = default ] && lib=structured_light_for_3d_model_replication_amd/libslgpu.so
    for cfg in "c5" "c2 --xyz exact"; do
      SLGPU_LIB=$(realpath $lib) timeout -k 10 200 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > $O/b.json 2>/dev/null || exit 1
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('$label'.ljust(8), '$cfg'.ljust(16), 'us/step %.1f'%(d['ms_per_step']*1e3), 'path %.3f'%d['roofline']['frac'], {k: round(v*1e3,1) for k,v in d['path']['rerun_ms_last_group'].items() if isinstance(v,float)})"
    done
  done
done
