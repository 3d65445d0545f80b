# Round 3: kernel timestamps of the c2 bench with and without --stack-ready
# (is k_stats beside the previous k_cloud, and what do the cross-stream waits
# cost?), then the exact k_cloud ablation kbench.  -> gpurun_out/r3tr, r3kc
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3tr
mkdir -p $O
for flag in --stack-ready --no-stack-ready; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$flag -o t -- python -u bench.py --steps 20 --warmup 5 --preroll-ms 30 --no-cpu-baseline --no-secondary $flag > $O/b$flag.json 2> $O/b$flag.err || { tail -20 $O/b$flag.err; exit 1; }
  f=$(find $O/t$flag -name '*kernel_trace.csv' | head -1)
  python3 scripts/trace_steps.py "$f" > $O/steps$flag.txt || exit 1
  rm -rf $O/t$flag
  tail -25 $O/steps$flag.txt
done
bash scripts/gpu_r3_kcloud_abl.sh "$@"
