# HIP API time of the merge stage (rocprofv3 --hip-trace --stats): where the host time goes
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/mh
mkdir -p $O
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python -u scripts/merge_bench.py --reps 3 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
f=$(find $O/trace -name '*hip_api_stats.csv' | head -1)
cp "$f" $O/hip_api_stats.csv
python3 - "$O/hip_api_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms  x{r["Calls"]:>6}  avg {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"]}')
PY
