#!/bin/bash
# Round 6: does the alignment of k_cloud's store windows to 128-B output lines
# matter?  step_floor with 800 points per chunk (every chunk's xyz region
# 128-B aligned) and 804 (unaligned), plain and aligned windows.
set -o pipefail
OUT=gpurun_out/${1:-r6_c}
mkdir -p "$OUT"
cd "$(dirname "$0")/.." || exit 1
echo "box: $(hostname) $(date -u +%FT%TZ)" > "$OUT/box.txt"
timeout -k 10 200 scripts/micro/step_floor --reps 3 --points 6480000 --variants cloud1,cloud1a,full,fulla > "$OUT/floor_ppc800.jsonl" 2>&1 &&
timeout -k 10 200 scripts/micro/step_floor --reps 3 --points 6512400 --variants cloud1,cloud1a,full,fulla > "$OUT/floor_ppc804.jsonl" 2>&1
rc=$?
echo "exit $rc" >> "$OUT/box.txt"
exit $rc
