#!/bin/bash
# Round 6: the graph-memset repro on torch's bundled HIP runtime (symlinked
# under its soname, so the standalone program loads it), the bench window's
# ramp (c2 at 20 vs 200 steps), and e2e over 8 folders per format.
set -o pipefail
OUT=gpurun_out/${1:-r6_e}
mkdir -p "$OUT"
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/torchhip && ln -sf "$TL/libamdhip64.so" /tmp/torchhip/libamdhip64.so.7
echo "box: $(hostname) $(date -u +%FT%TZ) torch_lib=$TL" > "$OUT/box.txt"
LD_LIBRARY_PATH=/tmp/torchhip ldd scripts/dbg/graph_memset | grep -E "amdhip|hsa" > "$OUT/ldd_torch_runtime.txt" &&
LD_LIBRARY_PATH=/tmp/torchhip timeout -k 10 120 scripts/dbg/graph_memset 6 > "$OUT/graph_memset_torch_runtime.jsonl" 2>&1 &&
timeout -k 10 120 scripts/dbg/graph_memset 6 > "$OUT/graph_memset_hip72.jsonl" 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --single-shot 0 > "$OUT/bench_c2_k20.json" 2> "$OUT/b.err" &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-secondary --single-shot 0 > "$OUT/bench_c2_k200.json" 2> "$OUT/b.err" &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --single-shot 0 > "$OUT/bench_c2_k20b.json" 2> "$OUT/b.err" &&
timeout -k 10 900 python -u scripts/e2e_bench.py --views 8 > "$OUT/e2e.jsonl" 2> "$OUT/e2e.err"
rc=$?
echo "exit $rc" >> "$OUT/box.txt"
exit $rc
