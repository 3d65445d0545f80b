"""HBM bytes per step (and per kernel launch) from rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes (separate runs) of a command that runs only the step's
kernels (scripts/kbench.py --only ...): 2*FETCH_SIZE (gfx950 tallies wide
coalesced reads at half, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KB
(x1024); each kernel launches once per step.

    python scripts/traffic_from_pmc.py <fetch_dir> <write_dir> <config> <views> <xyz fast|exact> <decide 0|1> <out.json>
"""
import csv
import glob
import json
import re
import sys


def per_kernel(d, counter):
    acc = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(k_\w+<[^>]*>|k_\w+)\(", r["Kernel_Name"])
            if m:
                acc.setdefault(m.group(1), []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
cfg, views, xyz, decide, out = sys.argv[3], int(sys.argv[4]), sys.argv[5], sys.argv[6] == "1", sys.argv[7]
kern = {k: (2 * fetch.get(k, 0.0) + write.get(k, 0.0)) * 1024 for k in sorted(set(fetch) | set(write))}
short = {}
for k, v in kern.items():
    short[k.split("<")[0]] = short.get(k.split("<")[0], 0.0) + v
res = {
    "config": cfg, "views": views, "xyz": xyz, "decide": decide,
    "bytes_per_step": sum(kern.values()),
    "kernels": short,
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over scripts/kbench.py "
              "(one output mode: every k_* kernel launch belongs to the step); HBM bytes = (2*FETCH_SIZE + "
              "WRITE_SIZE) KB * 1024 per launch (gfx950 half-count correction for wide reads, "
              "MI355X_MICROARCH.md HBM; WRITE_SIZE is calibrated for 16-B stores only -- k_cloud's 4-B / 1-B "
              "point stores are uncalibrated)",
    "per_kernel_KB": {k: {"FETCH_SIZE": fetch.get(k), "WRITE_SIZE": write.get(k)} for k in kern},
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
