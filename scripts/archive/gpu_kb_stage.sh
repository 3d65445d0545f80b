# k_cloud output staging A/B: default (direct per-point stores) vs
# SLGPU_STAGE_OUT=1 (lane-consecutive dword/byte stores) vs =2 (16-byte
# stores of the aligned middle): GPU tests on the =2 build, then kbench at
# config 2 (fast + exact) and a config-3-like batch (8 x 1920x1080).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/kst
mkdir -p $O
SLGPU_LIB=$PWD/build/libslgpu_swp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fast_f32.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_st2.log 2>&1 || { tail -30 $O/pytest_st2.log; exit 1; }
tail -1 $O/pytest_st2.log
: > $O/kb.log
for v in addr swp swpnost; do
  lib=structured_light_for_3d_model_replication_amd/libslgpu.so
  [ $v != default ] && lib=build/libslgpu_$v.so
  for args in "--fast --only cloud" "--fast --only cloud --views 8 --H 1080 --W 1920" "--fast --only maps+cloud"; do
    SLGPU_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/kbench.py --reps 30 $args | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$v $args\"/" >> $O/kb.log 2>&1 || exit 1
  done
done
grep variant $O/kb.log | grep -v torch_copy | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['lib'][:60].ljust(60), 'decode %.1f'%d['decode_us'], 'stats %.1f'%d['count_us'], 'cloud %.1f'%d['cloud_us'], 'wall %.1f'%d['wall_us_per_call'])"
