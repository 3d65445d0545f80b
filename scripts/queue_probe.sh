#!/bin/bash
# Which hardware queue each lane's kernels run on (rocprofv3 kernel-trace
# Queue_Id) for bench.py's lanes, per config.  -> gpurun_out/OUT/
set -o pipefail
OUT=gpurun_out/${1:-r6_q}
shift
mkdir -p "$OUT"
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
for cfg in "$@"; do
  IFS=':' read -r c streams <<< "$cfg"
  extra=""
  [ -n "$streams" ] && extra="--streams $streams"
  rm -rf "$OUT/tr"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o t -- python3 bench.py --config $c $extra \
    --steps 12 --warmup 3 --preroll-ms 20 --no-cpu-baseline --no-secondary --single-shot 0 > "$OUT/b_$c$streams.json" 2> "$OUT/b.err" || exit 1
  f=$(find "$OUT/tr" -name "*kernel_trace.csv" | head -1)
  python3 - "$f" "$c$streams" >> "$OUT/queues.jsonl" <<'PY' || exit 1
import csv, collections, json, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_decode" in r["Kernel_Name"] or "k_cloud" in r["Kernel_Name"]]
c = collections.Counter((r["Stream_Id"], r["Queue_Id"]) for r in rows)
print(json.dumps({"config": sys.argv[2], "stream_queue_dispatches": {f"{s}->{q}": n for (s, q), n in sorted(c.items())}}))
PY
  rm -rf "$OUT/tr"
done
cat "$OUT/queues.jsonl"
