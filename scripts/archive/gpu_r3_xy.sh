# Round 3: computed ray x / y in the exact k_cloud (xy_of, verified per table
# entry by sl_set_calib) -- the GPU parity subset, then the kbench A/B against
# the gathered tables (xy0) and the 1-KB plane-table ablation.  -> gpurun_out/r3xy, r3kc
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3xy
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_api_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash scripts/gpu_r3_kcloud_abl.sh "$@"
