#!/bin/bash
# Round 6: the whole-step floor and the graph-memset repro
# (#2) on one box, beside the bench's own c2 / c5 lines at HEAD.
#   scripts/gpu_r6_floor.sh OUT   (-> gpurun_out/OUT/)
set -o pipefail
OUT=gpurun_out/${1:-r6_floor}
mkdir -p "$OUT"
cd "$(dirname "$0")/.." || exit 1
echo "box: $(hostname) $(date -u +%FT%TZ)" > "$OUT/box.txt"
timeout -k 10 120 scripts/dbg/graph_memset 6 > "$OUT/graph_memset.jsonl" 2>&1 &&
timeout -k 10 180 python scripts/dbg/graph_memset_torch.py 6 > "$OUT/graph_memset_torch.jsonl" 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" &&
timeout -k 10 180 scripts/micro/step_floor --reps 3 --points 6455509 --variants full,no_pre,no_rec,bare,lanes1,chain,decode,cloud,mix > "$OUT/floor_c2.jsonl" 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_c2_b.json" 2> "$OUT/bench_c2_b.err" &&
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
timeout -k 10 300 scripts/micro/step_floor --read 24 --maps 0 --views 45 --group 8 --ring 1 --lanes 2 --points 6530219 \
  --steps 10 --warmup 3 --reps 2 --variants full,no_pre,no_rec,bare,lanes1,chain,mix > "$OUT/floor_c5.jsonl" 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_prestats.py -x -v --timeout 300 \
  --timeout-method thread > "$OUT/pytest_pool_prestats.log" 2>&1
rc=$?
echo "exit $rc" >> "$OUT/box.txt"
exit $rc
