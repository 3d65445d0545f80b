# Round 3: k_decode cross-group prefetch (SLGPU_DECODE_PF) at 2 waves per SIMD
# vs the default (no prefetch, 3 per SIMD): kbench re-runs, cloud-only 4 x
# 4000x3000 and 8 x 1080p, maps + cloud 4K.  Args: variants.  -> gpurun_out/r3pf
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3pf
mkdir -p $O
: > $O/kb.log
for rep in 1 2; do
  for v in default "$@"; do
    L=structured_light_for_3d_model_replication_amd/libslgpu.so
    [ $v != default ] && L=build/libslgpu_$v.so
    SLGPU_LIB=$(realpath $L) timeout -k 10 120 python -u scripts/kbench.py --H 3000 --W 4000 --views 4 --reps 20 --preroll-ms 300 --only cloud 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"$v c4x4\", /" >> $O/kb.log
    SLGPU_LIB=$(realpath $L) timeout -k 10 120 python -u scripts/kbench.py --H 1080 --W 1920 --views 8 --reps 20 --preroll-ms 300 --only cloud 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"$v c3x8\", /" >> $O/kb.log
    SLGPU_LIB=$(realpath $L) timeout -k 10 120 python -u scripts/kbench.py --reps 20 --preroll-ms 300 --only maps+cloud 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"$v c2\", /" >> $O/kb.log
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
for l in open('gpurun_out/r3pf/kb.log'):
    d = json.loads(l)
    rows[d['label']].append(d)
for lab, ds in sorted(rows.items(), key=lambda t: (t[0].split()[1], t[0])):
    g = lambda k: ' '.join('%.1f' % d['rerun_us'][k] for d in ds)
    print(lab.ljust(14), '| rerun decode', g('decode'), '| rerun cloud', g('cloud'), '| wall', ' '.join('%.1f' % d['wall_us_per_call'] for d in ds))
PY
