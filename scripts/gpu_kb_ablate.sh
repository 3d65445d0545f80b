# k_cloud / k_decode ablations via SLGPU_DEBUG (measurement only); args = dbg values
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/kbench.log
for d in "${@:-0}"; do
  SLGPU_DEBUG=$d timeout -k 10 120 python -u scripts/kbench.py --reps 20 >> gpurun_out/kbench.log 2>&1 || exit $?
done
grep -E "variant" gpurun_out/kbench.log
