"""Per-step timeline of a rocprofv3 --kernel-trace CSV of bench.py (measurement
helper): steps are delimited by k_decode launches; for each step, k_stats /
k_decode / k_cloud start and end relative to the step's k_decode start, and
the overlap of the step's k_stats with the previous step's k_cloud.

    python scripts/trace_steps.py <kernel_trace.csv> [last_n]
"""
import csv
import statistics as st
import sys


def main():
    path = sys.argv[1]
    last_n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    rows = [r for r in csv.DictReader(open(path)) if "k_" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def kind(r):
        n = r["Kernel_Name"]
        for k in ("k_stats", "k_decode", "k_cloud", "k_count"):
            if k in n:
                return k
        return "other"

    ev = [(kind(r), int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3, r.get("Queue_Id", "?"))
          for r in rows]
    decs = [i for i, e in enumerate(ev) if e[0] == "k_decode"]
    steps = []
    for j, i in enumerate(decs):
        d = ev[i]
        # this step's k_stats: the latest k_stats that started before this k_decode
        s = next((ev[k] for k in range(i - 1, -1, -1) if ev[k][0] == "k_stats"), None)
        c = next((ev[k] for k in range(i + 1, len(ev)) if ev[k][0] == "k_cloud"), None)
        prev_c = next((ev[k] for k in range(i - 1, -1, -1) if ev[k][0] == "k_cloud"), None)
        if s is None or c is None or prev_c is None:
            continue
        steps.append(dict(
            stats_us=s[2] - s[1], decode_us=d[2] - d[1], cloud_us=c[2] - c[1],
            stats_start=s[1] - prev_c[1], stats_end=s[2] - prev_c[1], prev_cloud_end=prev_c[2] - prev_c[1],
            gap_cloud_to_decode=d[1] - prev_c[2], gap_stats_to_decode=d[1] - s[2], gap_decode_to_cloud=c[1] - d[2],
            span=c[2] - prev_c[2], q=(s[3], d[3], c[3])))
    steps = steps[-last_n:]
    if not steps:
        print("no steps found")
        return
    print(f"{len(steps)} steps (the last {last_n}); times in us; 'rel' = relative to the previous step's k_cloud start")
    for k in ("stats_us", "decode_us", "cloud_us", "stats_start", "stats_end", "prev_cloud_end",
              "gap_cloud_to_decode", "gap_stats_to_decode", "gap_decode_to_cloud", "span"):
        v = [s[k] for s in steps]
        print(f"{k:22s} median {st.median(v):8.2f}  min {min(v):8.2f}  max {max(v):8.2f}")
    print("queues (stats, decode, cloud) of the last step:", steps[-1]["q"])
    for s in steps[-8:]:
        print("  ", " ".join(f"{k}={s[k]:.1f}" for k in ("stats_start", "stats_end", "prev_cloud_end",
                                                          "gap_cloud_to_decode", "span")))


if __name__ == "__main__":
    main()
