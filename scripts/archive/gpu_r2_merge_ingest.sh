# all GPU tests, merge bench (+ normals) with its rocprofv3 stats,
# and host ingest throughput on the box's core share -> gpurun_out/r2e
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r2e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash scripts/gpu_merge_prof.sh || exit 1
timeout -k 10 400 python -u scripts/ingest_bench.py --out $O/ingest_box.jsonl > $O/ingest.log 2>&1 || { tail -20 $O/ingest.log; exit 1; }
tail -3 $O/ingest.log
