# quick iteration: GPU parity tests + kernel bench (SLGPU_DEBUG values as args)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > gpurun_out/kbench.log
for d in "${@:-0}"; do
  SLGPU_DEBUG=$d timeout -k 10 120 python -u scripts/kbench.py >> gpurun_out/kbench.log 2>&1 || exit $?
done
grep -E "variant" gpurun_out/kbench.log | grep -v torch
exit $rc
