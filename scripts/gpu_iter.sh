# quick iteration: GPU parity tests + kernel bench over build variants
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > gpurun_out/kbench.log
for lib in "" build/libslgpu_occ3.so build/libslgpu_occ4.so; do
  [ -n "$lib" ] && [ ! -f "$lib" ] && continue
  echo "lib=$lib" >> gpurun_out/kbench.log
  SLGPU_LIB=$lib timeout -k 10 120 python -u scripts/kbench.py "$@" >> gpurun_out/kbench.log 2>&1 || exit $?
done
grep -E "variant|lib=" gpurun_out/kbench.log
exit $rc
