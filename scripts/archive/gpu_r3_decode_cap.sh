# Round 3: k_decode grid cap for cloud-only launches (4 x 4000x3000, the c4
# shape; and 8 x 1920x1080): SLGPU_DECODE_PER_CU = 0 (uncapped) / 2 / 3 / 4.  -> gpurun_out/r3cap
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3cap
mkdir -p $O
: > $O/kb.log
for rep in 1 2; do
  for cap in 3 0 2 4; do
    SLGPU_DECODE_PER_CU=$cap timeout -k 10 120 python -u scripts/kbench.py --H 3000 --W 4000 --views 4 --reps 20 --preroll-ms 300 --only cloud 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"cap$cap c4x4\", /" >> $O/kb.log
    SLGPU_DECODE_PER_CU=$cap timeout -k 10 120 python -u scripts/kbench.py --H 1080 --W 1920 --views 8 --reps 20 --preroll-ms 300 --only cloud 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"cap$cap c3x8\", /" >> $O/kb.log
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
for l in open('gpurun_out/r3cap/kb.log'):
    d = json.loads(l)
    rows[d['label']].append(d)
for lab, ds in sorted(rows.items()):
    g = lambda k: ' '.join('%.1f' % d['rerun_us'][k] for d in ds)
    print(lab.ljust(12), '| rerun decode', g('decode'), '| rerun cloud', g('cloud'), '| wall', ' '.join('%.1f' % d['wall_us_per_call'] for d in ds))
PY
