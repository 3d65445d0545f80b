# cost of the per-wave threshold computation in k_decode (ablation: constant thresholds)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/kthr
mkdir -p $O
SLGPU_LIB=$PWD/build/libslgpu_thr0.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/kb.log
for v in cur nothr thr0; do
  for args in "--fast --only maps+cloud" "--fast --only cloud"; do
    SLGPU_LIB=$PWD/build/libslgpu_$v.so timeout -k 10 120 python -u scripts/kbench.py --reps 50 $args | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$v $args\"/" >> $O/kb.log 2>&1 || exit 1
  done
done
grep variant $O/kb.log | grep -v torch_copy | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['lib'][:40].ljust(40), 'decode %.1f'%d['decode_us'], 'stats %.1f'%d['count_us'], 'cloud %.1f'%d['cloud_us'], 'wall %.1f'%d['wall_us_per_call'])"
