# Round-2 check: GPU tests, then the C2 bench on the single pass and on the
# three-kernel path (SLGPU_PATH=3), then a rocprofv3 kernel trace of the bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 4 > $O/bench_fused.json 2> $O/bench_fused.err || exit $?
tail -c 600 $O/bench_fused.json
SLGPU_PATH=3 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_3k.json 2> $O/bench_3k.err || exit $?
APP="python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- $APP > $O/trace.log 2>&1 || exit $?
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.2f} us  x{r["Calls"]:>4}  {r["Name"][:70]}')
PY
exit $rc
