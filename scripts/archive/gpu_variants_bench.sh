# build variants in build/ (libslgpu_o*.so): GPU parity tests with each, then kernel bench + bench.py c2
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/vb.log
for lib in build/libslgpu_o*.so; do
  SLGPU_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fast_f32.py -x -q --timeout 200 --timeout-method thread > gpurun_out/vb_pytest.log 2>&1 || { echo "parity FAILED with $lib"; tail -20 gpurun_out/vb_pytest.log; exit 1; }
  echo "lib=$lib parity ok" | tee -a gpurun_out/vb.log
done
for rep in 1 2; do
for lib in build/libslgpu_o*.so; do
  echo "lib=$lib" >> gpurun_out/vb.log
  SLGPU_LIB=$lib timeout -k 10 120 python -u scripts/kbench.py --reps 20 --only maps+cloud >> gpurun_out/vb.log 2>&1 || exit 1
  for cfg in ${CFGS:-c2}; do
  SLGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/vb_bench.json 2>/dev/null || exit 1
  python3 - $cfg >> gpurun_out/vb.log <<'PY'
import json, sys
d = json.loads(open("gpurun_out/vb_bench.json").read().strip().splitlines()[-1])
alt = d["alt_xyz_mode"]
print("bench", sys.argv[1], round(d["value"] / 1e9, 2), "Gpx/s", round(d["ms_per_step"] * 1e3, 1), "us", {k: round(v * 1e3, 1) for k, v in d["path"]["kernel_avg_ms"].items()}, "alt", alt and round(alt["k_cloud_ms"] * 1e3, 1))
PY
  done
done
done
grep -E "lib=|variant|bench" gpurun_out/vb.log | grep -v torch | cut -c1-250
