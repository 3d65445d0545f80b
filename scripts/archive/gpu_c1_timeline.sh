# config-1 timeline: rocprofv3 kernel trace of the bench, then per-step kernel
# durations and the gaps between them (is the step GPU- or host-bound?)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c1t
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o trace -- python -u bench.py --config c1 --steps 50 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, statistics as st
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'].split('(')[0].split('::')[-1][:12] for r in rows]
dur = {}
gaps = []
for i, r in enumerate(rows):
    n = names[i]
    dur.setdefault(n, []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    if i:
        gaps.append(((names[i-1], n), (int(r['Start_Timestamp']) - int(rows[i-1]['End_Timestamp'])) / 1e3))
for n, v in dur.items():
    print(f"{n:14s} n={len(v):4d} median {st.median(v):7.2f} us")
g = {}
for k, v in gaps:
    g.setdefault(k, []).append(v)
for k, v in g.items():
    print(f"gap {k[0]:>12s} -> {k[1]:12s} n={len(v):4d} median {st.median(v):7.2f} us  p90 {sorted(v)[int(0.9*len(v))]:7.2f}")
PY
tail -c 300 $O/bench.json
