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


def report(ev, label):
    t0 = min(x[1] for x in ev)
    span = max(x[2] for x in ev) - t0
    qs = {}
    for x in ev:
        qs[x[3]] = qs.get(x[3], 0) + 1
    by = {}
    for k, s, e, _, _ in ev:
        by.setdefault(k, []).append((s, e))
    ssum = sum(e - s for _, s, e, _, _ in ev)
    allb = union([(x[1], x[2]) for x in ev])
    dc = intersect(by.get("k_decode", []), by.get("k_cloud", []))
    kinds = "  ".join(f"{k} n={len(iv)} avg={sum(e - s for s, e in iv) / len(iv):.1f}" for k, iv in sorted(by.items()))
    print(f"{label}: span {span:.0f} us, busy {allb:.0f}, decode||cloud {dc:.0f}, sum/busy {ssum / allb:.3f}, "
          f"queues {dict(sorted(qs.items()))}  {kinds}")


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_" in r["Kernel_Name"]]
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    ev = []
    for r in rows:
        n = r["Kernel_Name"]
        k = next((k for k in ("k_stats", "k_decode", "k_cloud", "k_count", "k_fused") if k in n), "other")
        ev.append((k, int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3,
                   r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
    ev.sort(key=lambda x: x[1])
    # consecutive windows of `win` ms over the whole run (idle gaps > 5 ms
    # start a new window): the timed window is the multi-queue stretch
    cur = [ev[0]]
    for x in ev[1:]:
        if x[1] - cur[0][1] > win * 1e3 or x[1] - max(y[2] for y in cur[-4:]) > 5e3:
            report(cur, f"[{(cur[0][1] - ev[0][1]) / 1e3:8.1f} ms]")
            cur = []
        cur.append(x)
    report(cur, f"[{(cur[0][1] - ev[0][1]) / 1e3:8.1f} ms]")


if __name__ == "__main__":
    main()
