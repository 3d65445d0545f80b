# Parity (all GPU tests), then kbench --fast for the default path and the
# three-kernel path (SLGPU_PATH=3), maps+cloud and cloud.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/kab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > $O/kb.log
for only in "maps+cloud" "cloud"; do
  timeout -k 10 120 python -u scripts/kbench.py --reps 20 --fast --only "$only" >> $O/kb.log 2>&1 || exit $?
  SLGPU_PATH=3 timeout -k 10 120 python -u scripts/kbench.py --reps 20 --fast --only "$only" | sed 's/"lib": "libslgpu.so"/"lib": "3k"/' >> $O/kb.log 2>&1 || exit $?
done
grep variant $O/kb.log | grep -v torch_copy | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'][:10].ljust(10), d['lib'][:22].ljust(22), 'decode %.1f'%d['decode_us'], 'count/stats %.1f'%d['count_us'], 'cloud %.1f'%d['cloud_us'], 'wall %.1f'%d['wall_us_per_call'])"
