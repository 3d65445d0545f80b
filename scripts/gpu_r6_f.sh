#!/bin/bash
# Round 6: host ingest changes (colour file decoded beside the gray planes,
# per-plane H2D as planes land): the API / PLY GPU tests, then e2e over 8
# folders per format.  -> gpurun_out/OUT/
set -o pipefail
OUT=gpurun_out/${1:-r6_f}
mkdir -p "$OUT"
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
echo "box: $(hostname) $(date -u +%FT%TZ)" > "$OUT/box.txt"
timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_api_gpu.py \
  tests/test_gpu_ply_device.py tests/test_ply_io.py tests/test_ingest.py > "$OUT/pytest.log" 2>&1 &&
tail -1 "$OUT/pytest.log" &&
timeout -k 10 900 python -u scripts/e2e_bench.py --views 8 > "$OUT/e2e.jsonl" 2> "$OUT/e2e.err"
rc=$?
echo "exit $rc" >> "$OUT/box.txt"
exit $rc
