# k_decode grid cap sweep (SLGPU_DECODE_PER_CU = workgroups per CU, 0 = one
# workgroup per chunk group): parity tests under a capped grid, then kernel
# bench at config-2 and config-3 shapes per cap.
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && : > gpurun_out/decode_grid.log
SLGPU_DECODE_PER_CU=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/decode_grid_parity.log 2>&1 || { tail -20 gpurun_out/decode_grid_parity.log; exit 1; }
tail -1 gpurun_out/decode_grid_parity.log
for c in "$@"; do
  echo "per_cu=$c" >> gpurun_out/decode_grid.log
  SLGPU_DECODE_PER_CU=$c timeout -k 10 120 python -u scripts/kbench.py --reps 30 >> gpurun_out/decode_grid.log 2>&1 || exit $?
  SLGPU_DECODE_PER_CU=$c timeout -k 10 120 python -u scripts/kbench.py --H 1080 --W 1920 --views 8 --reps 30 --only cloud >> gpurun_out/decode_grid.log 2>&1 || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/decode_grid.log"):
    if l.startswith("per_cu"): print(l.strip())
    elif l.startswith("{") and "decode_us" in l:
        j = json.loads(l); print(f'  {j["variant"]:18s} decode {j["decode_us"]:7.1f} count {j["count_us"]:6.1f} cloud {j["cloud_us"]:6.1f} total {j["total_us"]:7.1f}')
PY
