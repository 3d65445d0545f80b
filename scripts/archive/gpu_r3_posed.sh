# Round 3: the verified route with a pose (c5's path) -- the full GPU suite,
# then c5 bench lines of this build vs the previous route (build/libslgpu_oldv.so)
# and c2 once more.  -> gpurun_out/r3posed
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3posed
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
: > $O/lines.log
for rep in 1 2; do
  for lib in default oldv; do
    L=structured_light_for_3d_model_replication_amd/libslgpu.so
    [ $lib = oldv ] && L=build/libslgpu_oldv.so
    SLGPU_LIB=$(realpath $L) timeout -k 10 400 python -u bench.py --config c5 --views 8 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/c5_$lib$rep.json 2> $O/c5_$lib$rep.err || { tail -20 $O/c5_$lib$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/c5_$lib$rep.json').read().strip().splitlines()[-1])
print('c5 8 views', '$lib', 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'], {k: round(v*1e3,1) for k,v in d['path']['rerun_ms_last_group'].items() if isinstance(v,float)})
" | tee -a $O/lines.log
  done
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1])
t=d['timing']['step_us']
print('c2', 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'], 'ev med %.1f' % t['median'], 'alt', d['alt_xyz_mode']['ms_per_step'])
" | tee -a $O/lines.log
