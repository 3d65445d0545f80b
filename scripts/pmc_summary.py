"""Summarise rocprofv3 --pmc counter_collection CSVs under a directory: per
kernel, the average of each counter over its dispatches."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        if not m:
            continue
        acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    print("==", k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {sum(v) / len(v):16.1f}   (n={len(v)})")
