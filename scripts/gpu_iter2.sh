# GPU parity tests, then kernel bench over SLGPU_DEBUG values (args) and build/ variants
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
: > gpurun_out/kbench.log
for d in "${@:-0}"; do
  SLGPU_DEBUG=$d timeout -k 10 120 python -u scripts/kbench.py --reps 20 >> gpurun_out/kbench.log 2>&1 || exit $?
done
for lib in build/libslgpu_*.so; do
  [ -e "$lib" ] || continue
  echo "{\"lib\": \"$lib\"}" >> gpurun_out/kbench.log
  SLGPU_LIB=$lib timeout -k 10 120 python -u scripts/kbench.py --reps 20 >> gpurun_out/kbench.log 2>&1 || exit $?
done
grep -E "variant|lib" gpurun_out/kbench.log | grep -v torch_copy
exit $rc
