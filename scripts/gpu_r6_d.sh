#!/bin/bash
# Round 6: the graph-memset repro under both HIP runtimes (the system's 7.2
# and torch's bundled 7.0, which torch processes -- and libslgpu.so inside
# them -- use), the torch repro with the node's addresses, and e2e (BMP).
set -o pipefail
OUT=gpurun_out/${1:-r6_d}
mkdir -p "$OUT"
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
echo "box: $(hostname) $(date -u +%FT%TZ) torch_lib=$TL" > "$OUT/box.txt"
timeout -k 10 120 scripts/dbg/graph_memset 6 > "$OUT/graph_memset_hip72.jsonl" 2>&1 &&
LD_LIBRARY_PATH=$TL timeout -k 10 120 scripts/dbg/graph_memset 6 > "$OUT/graph_memset_torch_runtime.jsonl" 2>&1 &&
LD_LIBRARY_PATH=$TL ldd scripts/dbg/graph_memset | grep -E "amdhip|hsa" > "$OUT/ldd_torch_runtime.txt" &&
timeout -k 10 180 python scripts/dbg/graph_memset_torch.py 6 > "$OUT/graph_memset_torch.jsonl" 2>&1 &&
timeout -k 10 600 python -u scripts/e2e_bench.py --views 4 --formats bmp > "$OUT/e2e_bmp.jsonl" 2> "$OUT/e2e.err"
rc=$?
echo "exit $rc" >> "$OUT/box.txt"
exit $rc
