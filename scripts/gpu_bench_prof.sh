# Full bench line + rocprofv3 kernel-trace summary + PMC traffic of the same
# command; results under gpurun_out/bp (copy what is judged into profiles/).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/bp
mkdir -p $O
CFG="${1:-c2}"
timeout -k 10 300 python -u bench.py --config $CFG --steps 20 --warmup 5 --cpu-seconds 10 > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json
APP="python -u bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- $APP > $O/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- $APP > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- $APP > $O/write.log 2>&1 || exit $?
python3 scripts/traffic_from_pmc.py $O/fetch $O/write $CFG 1 $O/traffic.json > /dev/null
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.2f} us  x{r["Calls"]:>4}  {r["Name"][:70]}')
PY
echo done
