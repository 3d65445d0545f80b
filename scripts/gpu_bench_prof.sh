# full bench line + rocprofv3 kernel-trace summary + PMC traffic passes for k_decode
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/bp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 10 > gpurun_out/bp/bench.json 2> gpurun_out/bp/bench.err || exit $?
tail -1 gpurun_out/bp/bench.json
APP="python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bp/trace -o trace -- $APP > gpurun_out/bp/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/bp/fetch -o fetch -- $APP > gpurun_out/bp/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/bp/write -o write -- $APP > gpurun_out/bp/write.log 2>&1 || exit $?
echo done
