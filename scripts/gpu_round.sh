set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_kbench.sh || exit $?
bash scripts/gpu_prof.sh || exit $?
