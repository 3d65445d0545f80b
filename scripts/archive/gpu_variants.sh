# kernel bench across build variants in build/ (libslgpu_o<occ>_r<ring>.so)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/variants.log
for lib in build/libslgpu_o*.so; do
  echo "lib=$lib" >> gpurun_out/variants.log
  SLGPU_LIB=$lib timeout -k 10 120 python -u scripts/kbench.py --reps 10 >> gpurun_out/variants.log 2>&1 || exit $?
done
grep -E "lib=|variant" gpurun_out/variants.log | grep -v torch
