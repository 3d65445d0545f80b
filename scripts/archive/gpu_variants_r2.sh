# kbench (maps+cloud and cloud, 4K view) for the shipped library and each
# build/libslgpu_*.so variant; SLGPU_PATH=3 for the three-kernel path.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/var
mkdir -p $O
: > $O/variants.log
for only in "maps+cloud" "cloud"; do
  timeout -k 10 120 python -u scripts/kbench.py --reps 20 --only "$only" >> $O/variants.log 2>&1 || exit $?
  SLGPU_PATH=3 timeout -k 10 120 python -u scripts/kbench.py --reps 20 --only "$only" | sed 's/"lib": "libslgpu.so"/"lib": "3k"/' >> $O/variants.log 2>&1 || exit $?
  for lib in build/libslgpu_*.so; do
    SLGPU_LIB=$lib timeout -k 10 120 python -u scripts/kbench.py --reps 20 --only "$only" >> $O/variants.log 2>&1 || exit $?
  done
done
grep variant $O/variants.log | grep -v torch_copy
