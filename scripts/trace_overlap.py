"""How much the kernels of a multi-stream run overlap (measurement helper).

    python scripts/trace_overlap.py <kernel_trace.csv> [window_ms]

Takes the last `window_ms` (default 20) of k_* dispatches of a rocprofv3
--kernel-trace CSV and prints, per kernel kind, the dispatches, summed
duration and busy time (union of its intervals), then the window's busy time
(union over all kinds), the time k_decode and k_cloud dispatches run at the
same moment, and the serial sum / union ratio (1.0 = no overlap at all).
"""
import csv
import sys


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0.0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def intersect(a, b):
    a, b = sorted(a), sorted(b)
    i = j = 0
    tot = 0.0
    # merge each list first
    def merged(v):
        out = []
        for s, e in v:
            if out and s <= out[-1][1]:
                out[-1][1] = max(out[-1][1], e)
            else:
                out.append([s, e])
        return out
    a, b = merged(a), merged(b)
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_" in r["Kernel_Name"]]
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    ev = []
    for r in rows:
        n = r["Kernel_Name"]
        k = next((k for k in ("k_stats", "k_decode", "k_cloud", "k_count", "k_fused") if k in n), "other")
        ev.append((k, int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3,
                   r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
    end = max(x[2] for x in ev)
    ev = [x for x in ev if x[1] >= end - win * 1e3]
    t0 = min(x[1] for x in ev)
    qs = {}
    for x in ev:
        qs[(x[3], x[4])] = qs.get((x[3], x[4]), 0) + 1
    print("dispatches by (queue, stream):", dict(sorted(qs.items())))
    span = end - t0
    print(f"window {span:.1f} us, {len(ev)} dispatches")
    by = {}
    for k, s, e, _, _ in ev:
        by.setdefault(k, []).append((s, e))
    ssum = 0.0
    for k, iv in sorted(by.items()):
        d = sum(e - s for s, e in iv)
        ssum += d
        print(f"  {k:9s} n={len(iv):4d}  sum {d:9.1f} us  busy {union(iv):9.1f} us  avg {d / len(iv):8.2f} us")
    allb = union([(x[1], x[2]) for x in ev])
    dc = intersect(by.get("k_decode", []), by.get("k_cloud", []))
    print(f"  busy (any kernel) {allb:.1f} us of {span:.1f}; decode||cloud {dc:.1f} us; sum/busy {ssum / allb:.3f}")


if __name__ == "__main__":
    main()
