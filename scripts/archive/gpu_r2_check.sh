# Round-2 check: all GPU tests, then the default bench line (C2) with its
# rocprofv3 kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -4 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 6 > $O/bench.json 2> $O/bench.err || exit $?
tail -c 1500 $O/bench.json
exit $rc
