# Round 3: where the exact (f64) k_cloud's time goes at config 2.  kbench
# (maps+cloud, C2 shape, 300 ms pre-roll) per measurement-only build in
# build/ (scripts/build_variants.sh), interleaved twice; "fast" = the in-tree
# library in SL_XYZ_F32_FAST for reference.  Args: variant names (build/
# libslgpu_<name>.so; "default" = in-tree).  -> gpurun_out/r3kc
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3kc
mkdir -p $O
: > $O/kb.log
for rep in 1 2; do
  for name in "$@" fast; do
    lib=structured_light_for_3d_model_replication_amd/libslgpu.so
    extra=""
    case $name in
      default) ;;
      fast) extra="--fast" ;;
      *) lib=build/libslgpu_$name.so ;;
    esac
    SLGPU_LIB=$(realpath $lib) timeout -k 10 120 python -u scripts/kbench.py --reps 30 --preroll-ms 300 --only maps+cloud $extra 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"$name\", /" >> $O/kb.log || { echo "kbench $name failed"; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
for l in open('gpurun_out/r3kc/kb.log'):
    d = json.loads(l)
    rows[d['label']].append(d)
for lab, ds in rows.items():
    f = lambda k: ' '.join('%.1f' % d[k] for d in ds)
    g = lambda k: ' '.join('%.1f' % d['rerun_us'][k] for d in ds)
    print(lab.ljust(8), 'stats', f('count_us'), '| decode', f('decode_us'), '| cloud', f('cloud_us'), '| rerun cloud', g('cloud'), '| wall', f('wall_us_per_call'))
PY
