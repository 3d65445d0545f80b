# GPU tests, then the default bench command itself under rocprofv3
# --kernel-trace --stats (the kernel averages must agree with the bench line's
# live HIP-event timings), then the plain bench line.  Results under
# gpurun_out/r2b (copy what is judged into profiles/).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r2b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -4 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python -u bench.py --steps 20 --warmup 5 --cpu-seconds 4 > $O/bench_traced.json 2> $O/bench_traced.err || exit $?
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/bench_kernel_stats.csv
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
tail -c 1500 $O/bench.json
exit $rc
