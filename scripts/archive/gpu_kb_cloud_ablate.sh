set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/kca
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/kb.log
for v in default cnostore cnomath cnogather cloadonly; do
  lib=structured_light_for_3d_model_replication_amd/libslgpu.so
  [ $v != default ] && lib=build/libslgpu_$v.so
  SLGPU_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/kbench.py --reps 30 --fast --only cloud | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$v\"/" >> $O/kb.log 2>&1 || exit 1
  SLGPU_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/kbench.py --reps 30 --only cloud | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$v exact\"/" >> $O/kb.log 2>&1 || exit 1
done
grep variant $O/kb.log | grep -v torch_copy | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['lib'][:18].ljust(18), 'decode %.1f'%d['decode_us'], 'stats %.1f'%d['count_us'], 'cloud %.1f'%d['cloud_us'], 'wall %.1f'%d['wall_us_per_call'])"
