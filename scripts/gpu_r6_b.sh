#!/bin/bash
# Round 6, second evidence call: k_cloud ablations at c2 (measurement builds
# build/libslgpu_<name>.so, scripts/build_variants.sh), config 1's kernels
# attributed (kernel trace + SQ counter passes, one lane and three), and the
# user-visible end-to-end rate (scripts/e2e_bench.py).  -> gpurun_out/OUT/
set -o pipefail
OUT=gpurun_out/${1:-r6_b}
mkdir -p "$OUT"
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
echo "box: $(hostname) $(date -u +%FT%TZ)" > "$OUT/box.txt"
: > "$OUT/kcloud_ablate.jsonl"
for rep in 1 2; do
  for v in abl0 gath arith prefix col xyz colxyz allbut; do
    SLGPU_LIB=$(realpath build/libslgpu_$v.so) timeout -k 10 120 python -u scripts/kbench.py --reps 30 --preroll-ms 300 \
      --only "maps+cloud" 2> "$OUT/kb.err" | grep '"maps+cloud"' | sed "s/^{/{\"abl\": \"$v\", \"rep\": $rep, /" >> "$OUT/kcloud_ablate.jsonl" || exit 1
  done
done
echo "ablations done" >> "$OUT/box.txt"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c1_l1" -o c1 -- \
  python3 -u scripts/steps_app.py --config c1 --lanes 1 --steps 200 > "$OUT/c1_l1.log" 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c1_l3" -o c1 -- \
  python3 -u scripts/steps_app.py --config c1 --lanes 3 --steps 200 > "$OUT/c1_l3.log" 2>&1 || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
k=0
for P in "$P1" "$P2" "$P3"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/c1_pmc$k" -o p -- \
    python3 -u scripts/steps_app.py --config c1 --lanes 1 --steps 20 > "$OUT/c1_pmc$k.log" 2>&1 || exit 1
done
echo "c1 done" >> "$OUT/box.txt"
timeout -k 10 600 python -u scripts/e2e_bench.py --views 4 > "$OUT/e2e.jsonl" 2> "$OUT/e2e.err"
rc=$?
echo "exit $rc" >> "$OUT/box.txt"
exit $rc
