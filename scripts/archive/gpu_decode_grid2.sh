# k_decode grid cap (SLGPU_DECODE_PER_CU) on the cloud-only shapes of configs 2, 4, 5
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && : > gpurun_out/decode_grid2.log
for c in "$@"; do
  for shape in "--H 2160 --W 3840 --views 1" "--H 2160 --W 3840 --views 2" "--H 3000 --W 4000 --views 1"; do
    echo "per_cu=$c $shape" >> gpurun_out/decode_grid2.log
    SLGPU_DECODE_PER_CU=$c timeout -k 10 120 python -u scripts/kbench.py $shape --reps 50 --only cloud >> gpurun_out/decode_grid2.log 2>&1 || exit $?
  done
  echo "per_cu=$c maps+cloud" >> gpurun_out/decode_grid2.log
  SLGPU_DECODE_PER_CU=$c timeout -k 10 120 python -u scripts/kbench.py --reps 50 --only maps+cloud >> gpurun_out/decode_grid2.log 2>&1 || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/decode_grid2.log"):
    if l.startswith("per_cu"): print(l.strip(), end="")
    elif l.startswith("{") and "decode_us" in l:
        j = json.loads(l); print(f'   decode {j["decode_us"]:7.1f} count {j["count_us"]:6.1f} cloud {j["cloud_us"]:6.1f} total {j["total_us"]:7.1f}')
PY
