# rocprofv3 PMC passes (one counter group per run) over one kbench variant ($1);
# per-kernel averages printed.  HBM bytes: 2*FETCH_SIZE (gfx950 counts half of
# wide coalesced reads, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, in KB.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
V="${1:-maps+cloud}"
OUT=gpurun_out/pmc
mkdir -p $OUT
APP="python -u scripts/kbench.py --reps 5 --only $V"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_FLAT SQ_INST_CYCLES_VMEM_RD" \
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- $APP > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc; exit 0
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_" not in k: continue
        k = k.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print("==", k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {sum(v)/len(v):16.1f}")
PY
