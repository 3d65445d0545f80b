# merge-stage bench line + rocprofv3 kernel stats of it -> gpurun_out/mb
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/mb
mkdir -p $O
timeout -k 10 300 python -u scripts/merge_bench.py "$@" > $O/merge.json 2> $O/merge.err || { tail -20 $O/merge.err; exit 1; }
cat $O/merge.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python -u scripts/merge_bench.py --reps 1 "$@" > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{float(r["AverageNs"])/1e3:10.2f} us  x{r["Calls"]:>4}  tot {float(r["TotalDurationNs"])/1e6:8.2f} ms  {r["Name"][:60]}')
PY
