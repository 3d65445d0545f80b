# Round 3 same-box A/B of library builds on the exact (f64) path: per build,
# the parity subset (tests/test_gpu_parity.py), then kbench (exact, C2 shape,
# 300 ms pre-roll, HIP events + back-to-back re-runs) twice interleaved, then
# one bench.py c2 line.  Arguments: "label|lib[|ENV=V ...]" ("default" = in-tree).
# -> gpurun_out/r3ab
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3ab
mkdir -p $O
: > $O/kb.log
: > $O/bench.log
for spec in "$@"; do
  IFS='|' read -r label lib envs <<< "$spec"
  [ "$lib" = default ] && lib=structured_light_for_3d_model_replication_amd/libslgpu.so
  env ${envs:-} SLGPU_LIB=$(realpath $lib) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden_fused or golden_cloud or synthetic or full_4k or multiview" > $O/pytest_$label.log 2>&1 || { echo "parity FAILED for $label"; tail -30 $O/pytest_$label.log; exit 1; }
  echo "$label parity: $(tail -1 $O/pytest_$label.log)"
done
for rep in 1 2; do
  for spec in "$@"; do
    IFS='|' read -r label lib envs <<< "$spec"
    [ "$lib" = default ] && lib=structured_light_for_3d_model_replication_amd/libslgpu.so
    for only in ${AB_MODES:-"maps+cloud" "cloud"}; do
      env ${envs:-} SLGPU_LIB=$(realpath $lib) timeout -k 10 120 python -u scripts/kbench.py --reps 30 --preroll-ms 300 --only "$only" ${AB_KB:-} 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"$label\", /" >> $O/kb.log || exit 1
    done
  done
done
for spec in "$@"; do
  IFS='|' read -r label lib envs <<< "$spec"
  [ "$lib" = default ] && lib=structured_light_for_3d_model_replication_amd/libslgpu.so
  for cfg in ${AB_CONFIGS:-c2}; do
    env ${envs:-} SLGPU_LIB=$(realpath $lib) timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-secondary ${AB_BENCH:-} > $O/bench_${label}_$cfg.json 2> $O/bench_${label}_$cfg.err || { tail -20 $O/bench_${label}_$cfg.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$O/bench_${label}_$cfg.json').read().strip().splitlines()[-1])
t=d['timing']['step_us']
print('$label', '$cfg', 'ms/step %.4f'%d['ms_per_step'], 'Gpx/s %.1f'%(d['value']/1e9), 'frac %.3f'%d['roofline']['frac'], 'ev_median %.1f'%t['median'], {k: round(v*1e3,1) for k,v in d['path']['rerun_ms_last_group'].items() if isinstance(v,float)})
" | tee -a $O/bench.log
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
for l in open('gpurun_out/r3ab/kb.log'):
    d = json.loads(l)
    rows[(d['label'], d['variant'])].append(d)
for (lab, var), ds in rows.items():
    f = lambda k: ' '.join('%.1f' % d[k] for d in ds)
    g = lambda k: ' '.join('%.1f' % d['rerun_us'][k] for d in ds)
    print(lab[:10].ljust(10), var[:10].ljust(10), 'stats', f('count_us'), '| decode', f('decode_us'), '| cloud', f('cloud_us'), '| rerun cloud', g('cloud'), '| wall', f('wall_us_per_call'))
PY
