for lib in build/libslgpu_sp4.so build/libslgpu_sp8.so structured_light_for_3d_model_replication_amd/libslgpu.so build/libslgpu_sp4.so build/libslgpu_sp8.so structured_light_for_3d_model_replication_amd/libslgpu.so; do
  SLGPU_LIB=$(realpath $lib) timeout -k 10 200 python -u bench.py --config c1 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab/c1.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab/c1.json').read().strip().splitlines()[-1])
print('$lib'.split('/')[-1], 'c1 us/step %.1f'%(d['ms_per_step']*1e3), {k: round(v*1e3,1) for k,v in d['path']['rerun_ms_last_group'].items() if isinstance(v,float)})"
done
