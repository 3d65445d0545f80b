# Round-2 profile of the headline workload (C2, maps + f32-fast cloud):
# rocprofv3 kernel trace + stats, PMC FETCH_SIZE / WRITE_SIZE passes (separate
# runs, per MI355X_MICROARCH.md) -> per-step HBM bytes, then the bench line
# (which reads that traffic file).  Results under gpurun_out/prof (copy what
# is judged into profiles/).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
APP="python -u scripts/kbench.py --reps 10 --fast --only maps+cloud"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- $APP > $O/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- $APP > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- $APP > $O/write.log 2>&1 || exit $?
python3 scripts/traffic_from_pmc.py $O/fetch $O/write c2 1 fast 1 $O/traffic_c2.json > /dev/null || exit $?
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.2f} us  x{r["Calls"]:>4}  {r["Name"][:70]}')
PY
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 10 --traffic $O/traffic_c2.json > $O/bench.json 2> $O/bench.err || exit $?
tail -c 700 $O/bench.json
