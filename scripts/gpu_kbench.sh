set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for d in 0 1 3; do
  SLGPU_DEBUG=$d timeout -k 10 120 python -u scripts/kbench.py >> gpurun_out/kbench.log 2>&1 || exit $?
done
SLGPU_DEBUG=0 timeout -k 10 120 python -u scripts/kbench.py --views 4 >> gpurun_out/kbench.log 2>&1 || exit $?
grep variant gpurun_out/kbench.log
