# Round 3: k_stats with lane-private byte counters (default) vs the shared
# replicas (build/libslgpu_st0.so): the GPU parity file, kbench at c2 (maps +
# cloud) and at 4 x 4000x3000 cloud only, and a c3 line each.  -> gpurun_out/r3st
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3st
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_api_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/kb.log
for rep in 1 2; do
  for v in default st0; do
    L=structured_light_for_3d_model_replication_amd/libslgpu.so
    [ $v = st0 ] && L=build/libslgpu_st0.so
    SLGPU_LIB=$(realpath $L) timeout -k 10 120 python -u scripts/kbench.py --reps 30 --preroll-ms 300 --only maps+cloud 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"$v c2\", /" >> $O/kb.log
    SLGPU_LIB=$(realpath $L) timeout -k 10 120 python -u scripts/kbench.py --H 3000 --W 4000 --views 4 --reps 20 --preroll-ms 300 --only cloud 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"$v c4x4\", /" >> $O/kb.log
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
for l in open('gpurun_out/r3st/kb.log'):
    d = json.loads(l)
    rows[d['label']].append(d)
for lab, ds in rows.items():
    f = lambda k: ' '.join('%.1f' % d[k] for d in ds)
    g = lambda k: ' '.join('%.1f' % d['rerun_us'][k] for d in ds)
    print(lab.ljust(10), 'stats', f('count_us'), '| rerun stats', g('stats_count'), '| decode', f('decode_us'), '| cloud', f('cloud_us'), '| wall', f('wall_us_per_call'))
PY
for v in default st0; do
  L=structured_light_for_3d_model_replication_amd/libslgpu.so
  [ $v = st0 ] && L=build/libslgpu_st0.so
  SLGPU_LIB=$(realpath $L) timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > $O/c2_$v.json 2> $O/c2_$v.err || { tail -20 $O/c2_$v.err; exit 1; }
  SLGPU_LIB=$(realpath $L) timeout -k 10 300 python -u bench.py --config c3 --scaling strong --no-cpu-baseline --no-secondary > $O/c3_$v.json 2> $O/c3_$v.err || { tail -20 $O/c3_$v.err; exit 1; }
  for c in c2 c3; do
    python3 -c "
import json
d=json.loads(open('$O/${c}_$v.json').read().strip().splitlines()[-1])
print('$c $v', 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'])
"
  done
done
