# small-frame (config-1 size) kernel times: adaptive vs fixed mask (histogram atomics), then all configs' bench lines
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cfg
for v in "maps+cloud" "maps+cloud fixed"; do
  timeout -k 10 120 python -u scripts/kbench.py --H 720 --W 1280 --reps 50 --only "$v" 2>&1 | grep variant | grep -v torch || exit 1
done
for c in c1 c2 c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/cfg/$c.json 2> gpurun_out/cfg/$c.err || { tail -5 gpurun_out/cfg/$c.err; exit 1; }
done
