# Quick parity (tests/test_gpu_parity.py), then kbench --fast (maps+cloud and
# cloud) for the shipped library and every build/libslgpu_*.so variant.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/kbv
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > $O/kb.log
for only in "maps+cloud" "cloud"; do
  for lib in structured_light_for_3d_model_replication_amd/libslgpu.so build/libslgpu_*.so; do
    SLGPU_LIB=$(realpath $lib) timeout -k 10 120 python -u scripts/kbench.py --reps 20 --fast --only "$only" >> $O/kb.log 2>&1 || exit $?
  done
done
grep variant $O/kb.log | grep -v torch_copy | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'][:10].ljust(10), d['lib'][:22].ljust(22), 'decode %.1f'%d['decode_us'], 'count %.1f'%d['count_us'], 'cloud %.1f'%d['cloud_us'], 'wall %.1f'%d['wall_us_per_call'])"
