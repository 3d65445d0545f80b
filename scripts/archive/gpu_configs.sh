# bench.py over the BASELINE configs (args: config names), one JSON line each
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cfg
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/cfg/$c.json 2> gpurun_out/cfg/$c.err || { tail -20 gpurun_out/cfg/$c.err; exit 1; }
  tail -1 gpurun_out/cfg/$c.json
done
