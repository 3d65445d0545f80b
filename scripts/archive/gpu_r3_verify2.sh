# Round 3: the normalisation-free verified route (P' = v q') -- GPU parity
# (the verified-route tests vs the exact sequence, the golden / synthetic /
# full-4K parity cases), then kbench of the verify pipe widths against the
# previous route (oldv) and f32-fast.  -> gpurun_out/r3v2, r3kc
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3v2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fast_f32.py tests/test_gpu_pool.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in ${VARIANT_TESTS:-}; do
  SLGPU_LIB=$(realpath build/libslgpu_$v.so) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "verified or golden_fused or full_4k or synthetic" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
bash scripts/gpu_r3_kcloud_abl.sh "$@"
