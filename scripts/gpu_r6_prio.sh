#!/bin/bash
# Lane stream priority A/B (high-priority streams get hardware queues of their
# own): per rep, each (config, streams, priority) bench line alternating.
set -o pipefail
OUT=gpurun_out/${1:-r6_prio}
shift
mkdir -p "$OUT"
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
echo "box: $(hostname) $(date -u +%FT%TZ)" > "$OUT/box.txt"
: > "$OUT/lines.jsonl"
for rep in 1 2 3; do
  for spec in "$@"; do
    IFS=':' read -r cfg st pr <<< "$spec"
    timeout -k 10 300 python3 -u bench.py --config $cfg --streams $st --lane-priority $pr --no-cpu-baseline --no-secondary \
      --single-shot 0 > "$OUT/b.json" 2> "$OUT/b.err" || { tail -20 "$OUT/b.err"; exit 1; }
    tail -1 "$OUT/b.json" | sed "s/^{/{\"label\": \"$spec\", \"rep\": $rep, /" >> "$OUT/lines.jsonl"
  done
done
python3 - "$OUT/lines.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["label"], d["rep"], "us/step %.2f" % (1e3 * d["ms_per_step"]), "frac %.4f" % d["roofline"]["frac"], d["verified"])
PY
