# k_decode (decide path) ablations: per-iteration block-sum barrier, LDS table fill
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/kda
mkdir -p $O
: > $O/kb.log
for v in cur nobar nofill both; do
  for args in "--fast --only maps+cloud" "--fast --only cloud" "--fast --only cloud --views 4 --H 3000 --W 4000"; do
    SLGPU_LIB=$PWD/build/libslgpu_$v.so timeout -k 10 120 python -u scripts/kbench.py --reps 30 $args | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$v $args\"/" >> $O/kb.log 2>&1 || exit 1
  done
done
grep variant $O/kb.log | grep -v torch_copy | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['lib'][:62].ljust(62), 'decode %.1f'%d['decode_us'], 'stats %.1f'%d['count_us'], 'cloud %.1f'%d['cloud_us'], 'wall %.1f'%d['wall_us_per_call'])"
