# Round 3: the posed verified route's midpoint test (M_k <= 16 |v|) -- posed
# GPU tests, c5 A/B against build/libslgpu_head.so.  -> gpurun_out/r3posed2
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3posed2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pool.py -x -q --timeout 120 --timeout-method thread -k "pose or verified or posed" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/lines.log
for rep in 1 2; do
  for lib in default head; do
    L=structured_light_for_3d_model_replication_amd/libslgpu.so
    [ $lib = head ] && L=build/libslgpu_head.so
    SLGPU_LIB=$(realpath $L) timeout -k 10 400 python -u bench.py --config c5 --views 16 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/c5_$lib$rep.json 2> $O/c5_$lib$rep.err || { tail -20 $O/c5_$lib$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/c5_$lib$rep.json').read().strip().splitlines()[-1])
print('c5 16 views', '$lib', 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'], {k: round(v*1e3,1) for k,v in d['path']['rerun_ms_last_group'].items() if isinstance(v,float)})
" | tee -a $O/lines.log
  done
done
