"""How the lanes' kernels overlap in a rocprofv3 kernel trace of bench.py.

    python scripts/trace_lanes.py kernel_trace.csv [--last 150]

Takes the last ``--last`` k_decode / k_stats / k_cloud dispatches (the timed
window's tail), and prints per kernel its mean duration and count, then over
the span they cover: the busy time (union of the intervals), the kernel time
summed, their ratio (how many kernels run at once on average), the idle gaps,
and the histogram of concurrency (time with 0, 1, 2, ... kernels running).
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=150)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if not any(k in name for k in ("k_decode", "k_cloud", "k_stats")):
                continue
            kind = "k_decode" if "k_decode" in name else ("k_cloud" if "k_cloud" in name else "k_stats")
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, q))
    rows.sort()
    rows = rows[-a.last:]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    per = defaultdict(list)
    for s, e, k, _ in rows:
        per[k].append(e - s)
    ev = sorted([(s, 1) for s, *_ in rows] + [(e, -1) for _, e, *_ in rows])
    conc = defaultdict(int)
    cur, last = 0, t0
    for t, d in ev:
        conc[cur] += t - last
        cur += d
        last = t
    span = t1 - t0
    busy = span - conc.get(0, 0)
    total = sum(e - s for s, e, *_ in rows)
    queues = sorted({q for *_, q in rows})
    out = {
        "dispatches": len(rows), "queues": queues, "span_us": span / 1e3, "busy_us": busy / 1e3,
        "kernel_us_summed": total / 1e3, "mean_concurrency_when_busy": total / busy if busy else None,
        "idle_frac": conc.get(0, 0) / span if span else None,
        "time_at_concurrency_frac": {str(k): v / span for k, v in sorted(conc.items())},
        "per_kernel": {k: {"n": len(v), "mean_us": sum(v) / len(v) / 1e3} for k, v in per.items()},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
