set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python -u bench.py --config c1 --steps 50 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || exit 1
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/kernel_stats.csv
f2=$(find $O/trace -name '*kernel_trace.csv' | head -1)
cp "$f2" $O/kernel_trace.csv
tail -1 $O/trace.log | cut -c1-400
