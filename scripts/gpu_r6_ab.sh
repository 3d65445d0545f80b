#!/bin/bash
# Round 6 same-box A/B of library builds: the GPU parity suite on the shipped
# (in-tree) library first, then per rep and per build (alternating): kbench
# (c2 shape, maps + cloud and cloud; 300 ms pre-roll) and one bench line per
# config in $AB_CONFIGS.  Arguments: "label|lib" ("default" = in-tree).
# -> gpurun_out/$AB_OUT (default r6_ab)
set -u -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-r6_ab}
mkdir -p $O
echo "box: $(hostname) $(date -u +%FT%TZ)" > $O/box.txt
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $AB_TESTS -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
: > $O/kb.jsonl
: > $O/bench_lines.jsonl
for rep in $(seq 1 ${AB_REPS:-2}); do
  for spec in "$@"; do
    IFS='|' read -r label lib <<< "$spec"
    [ "$lib" = default ] && lib=structured_light_for_3d_model_replication_amd/libslgpu.so
    for only in ${AB_MODES:-"maps+cloud"}; do
      SLGPU_LIB=$(realpath $lib) timeout -k 10 120 python -u scripts/kbench.py --reps 30 --preroll-ms 300 --only "$only" 2>/dev/null \
        | grep '"variant"' | grep -v torch_copy | sed "s/^{/{\"label\": \"$label\", \"rep\": $rep, /" >> $O/kb.jsonl || exit 1
    done
    for cfg in ${AB_CONFIGS:-c2}; do
      SLGPU_LIB=$(realpath $lib) timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-secondary \
        --single-shot 0 ${AB_BENCH:-} > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      tail -1 $O/b.json | sed "s/^{/{\"label\": \"$label\", \"rep\": $rep, \"cfg\": \"$cfg\", /" >> $O/bench_lines.jsonl
    done
  done
done
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(f"{O}/kb.jsonl"):
    d = json.loads(l)
    print("kb", d["label"], d["rep"], d["variant"], "rerun", {k: round(v, 2) for k, v in d["rerun_us"].items()})
for l in open(f"{O}/bench_lines.jsonl"):
    d = json.loads(l)
    print("bench", d["label"], d["rep"], d["cfg"], "us/step %.2f" % (1e3 * d["ms_per_step"]), "frac %.4f" % d["roofline"]["frac"],
          "verified", d["verified"])
PY
