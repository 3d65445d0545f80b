# kernel-bench ablations (SLGPU_DEBUG values given as args) for one kbench variant
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && : > gpurun_out/kb_ablate.log
only=${ONLY:-maps+cloud}
for d in "$@"; do
  SLGPU_DEBUG=$d timeout -k 10 120 python -u scripts/kbench.py --reps 20 --only "$only" >> gpurun_out/kb_ablate.log 2>&1 || exit $?
done
grep variant gpurun_out/kb_ablate.log | grep -v torch
