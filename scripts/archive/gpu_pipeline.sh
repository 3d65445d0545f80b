# GPU tests + the host-resident pipeline bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u scripts/pipeline_bench.py --views 16 --files 2 > gpurun_out/pipeline.jsonl 2> gpurun_out/pipeline.err || { tail -20 gpurun_out/pipeline.err; exit 1; }
cat gpurun_out/pipeline.jsonl
