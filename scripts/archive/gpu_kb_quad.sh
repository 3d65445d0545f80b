# k_decode quad layout A/B: GPU tests on the quad build, then kbench
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/quad
mkdir -p $O
SLGPU_LIB=$PWD/build/libslgpu_quadw2.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/kb.log
for v in noquad quad quadw2 noquadw2; do
  for args in "--fast --only maps+cloud" "--fast --only cloud" "--fast --only cloud --views 4 --H 3000 --W 4000" "--fast --only maps+cloud --H 720 --W 1280"; do
    SLGPU_LIB=$PWD/build/libslgpu_$v.so timeout -k 10 120 python -u scripts/kbench.py --reps 30 $args | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$v $args\"/" >> $O/kb.log 2>&1 || exit 1
  done
done
grep variant $O/kb.log | grep -v torch_copy | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['lib'][:62].ljust(62), 'decode %.1f'%d['decode_us'], 'stats %.1f'%d['count_us'], 'cloud %.1f'%d['cloud_us'], 'wall %.1f'%d['wall_us_per_call'])"
