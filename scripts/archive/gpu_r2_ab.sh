# Same-box A/B of library variants with scripts/kbench.py (--fast, C2 shape):
# arguments are "label|ENV=VAL ...|lib" triples (lib: path or "default"); each
# variant runs twice, interleaved.  Optional GPU parity first (AB_TESTS=1) and
# extra commands after (AB_AFTER).  -> gpurun_out/ab
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
if [ "${AB_TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
: > $O/kb.log
for rep in 1 2; do
  for spec in "$@"; do
    IFS='|' read -r label envs lib <<< "$spec"
    [ "$lib" = default ] && lib=structured_light_for_3d_model_replication_amd/libslgpu.so
    for only in ${AB_MODES:-"maps+cloud" "cloud"}; do
      env $envs SLGPU_LIB=$(realpath $lib) timeout -k 10 120 python -u scripts/kbench.py --reps 30 --fast --only "$only" ${AB_SHAPE:-} 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"$label\", /" >> $O/kb.log || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
for l in open('gpurun_out/ab/kb.log'):
    d = json.loads(l)
    rows[(d['label'], d['variant'])].append(d)
for (lab, var), ds in rows.items():
    f = lambda k: ' '.join('%.1f' % d[k] for d in ds)
    print(lab[:16].ljust(16), var[:10].ljust(10), 'stats', f('count_us'), '| decode', f('decode_us'), '| cloud', f('cloud_us'), '| wall', f('wall_us_per_call'))
PY
if [ -n "${AB_AFTER:-}" ]; then bash -c "$AB_AFTER" || exit 1; fi
