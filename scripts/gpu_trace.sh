# rocprofv3 kernel trace of one kbench variant ($1, default maps+cloud) for each
# SLGPU_DEBUG value in $2.. (default 0); per-kernel averages printed
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
V="${1:-maps+cloud}"
shift || true
for d in "${@:-0}"; do
  out=gpurun_out/trace/d$d
  mkdir -p $out
  SLGPU_DEBUG=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/raw -o run -- python -u scripts/kbench.py --reps 20 --only "$V" > $out/log.txt 2>&1 || exit $?
  f=$(find $out/raw -name '*kernel_stats.csv' | head -1)
  cp "$f" $out/kernel_stats.csv
  echo "== SLGPU_DEBUG=$d variant=$V"
  python3 - "$out/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "k_" in n or "copyBuffer" in n:
        print(f'{float(r["AverageNs"])/1e3:9.2f} us  x{r["Calls"]:>4}  {n[:80]}')
PY
done
