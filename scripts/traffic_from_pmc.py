"""HBM bytes per step (and per kernel launch) from rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes (separate runs) of a command that runs only the step's
kernels (scripts/kbench.py --only ...): 2*FETCH_SIZE (gfx950 tallies wide
coalesced reads at half, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KB
(x1024); each kernel launches once per step.

    python scripts/traffic_from_pmc.py <fetch_dir> <write_dir> <config> <views> <xyz fast|exact> <decide 0|1> <out.json>
        [--calib <cal_fetch_dir> <cal_write_dir> <store_calib stdout json>] [--per-step N]

--per-step N (a command that runs N steps and nothing else, scripts/steps_app.py):
every kernel's bytes summed over its launches and divided by N, instead of
one average launch per kernel per step.
"""
import csv
import glob
import json
import re
import sys


STEP_KERNELS = ("k_stats", "k_decode", "k_count", "k_cloud")  # (sl_set_calib's k_xy_check is not a step's)


PER_STEP = None  # --per-step N


def per_kernel(d, counter):
    acc = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(k_\w+<[^>]*>|k_\w+)\(", r["Kernel_Name"])
            if m and m.group(1).split("<")[0] in STEP_KERNELS:
                acc.setdefault(m.group(1), []).append(float(r["Counter_Value"]))
    return {k: sum(v) / (PER_STEP or len(v)) for k, v in acc.items()}


def calib_factors(fdir, wdir, cal_json):
    """bytes per reported byte of each access shape of scripts/micro/store_calib
    (known byte counts; FETCH_SIZE / WRITE_SIZE in KB)."""
    known = json.loads(open(cal_json).read().strip().splitlines()[-1])["bytes"]

    def rep(d, counter):
        acc = {}
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == counter:
                    m = re.match(r"\s*(?:void\s+)?(\w+)\(", r["Kernel_Name"])
                    if m and m.group(1) in known:
                        acc.setdefault(m.group(1), []).append(float(r["Counter_Value"]) * 1024)
        return {k: sum(v) / len(v) for k, v in acc.items()}

    w, f = rep(wdir, "WRITE_SIZE"), rep(fdir, "FETCH_SIZE")
    fac = {}
    for k in ("st16", "st12", "st3", "pts"):
        if w.get(k):
            fac["write_" + k] = known[k] / w[k]
    for k in ("ld8", "ld16"):
        if f.get(k):
            fac["fetch_" + k] = known[k] / f[k]
    return fac


args = [a for a in sys.argv[1:]]
cal = None
if "--calib" in args:
    i = args.index("--calib")
    cal = calib_factors(args[i + 1], args[i + 2], args[i + 3])
    del args[i:i + 4]
if "--per-step" in args:
    i = args.index("--per-step")
    PER_STEP = int(args[i + 1])
    del args[i:i + 2]
RING = 1  # --ring R: the steps cycled through R distinct resident views (bench.py --ring)
if "--ring" in args:
    i = args.index("--ring")
    RING = int(args[i + 1])
    del args[i:i + 2]
fetch, write = per_kernel(args[0], "FETCH_SIZE"), per_kernel(args[1], "WRITE_SIZE")
cfg, views, xyz, decide, out = args[2], int(args[3]), args[4], args[5] == "1", args[6]
kern = {k: (2 * fetch.get(k, 0.0) + write.get(k, 0.0)) * 1024 for k in sorted(set(fetch) | set(write))}


def corrected(k):
    """Calibrated bytes of kernel k: its reads and writes by the factor of the
    access shapes it uses (k_cloud reads 8-B records and 16-B texture words in
    the algorithmic ratio 1.5 : 3 per pixel; its stores are the 12-B + 3-B
    point pattern; k_decode / k_stats: 16-B streaming reads, 16-B map stores)."""
    fr, wr = fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
    if k.startswith("k_cloud"):
        a8, a16 = 1.5, 3.0
        f8, f16 = cal.get("fetch_ld8", 2.0), cal.get("fetch_ld16", 2.0)
        ff = (a8 + a16) / (a8 / f8 + a16 / f16)
        return fr * ff + wr * cal.get("write_pts", 1.0)
    return fr * cal.get("fetch_ld16", 2.0) + wr * cal.get("write_st16", 1.0)


short = {}
kern_use = {k: corrected(k) for k in kern} if cal else kern
for k, v in kern_use.items():
    short[k.split("<")[0]] = short.get(k.split("<")[0], 0.0) + v
res = {
    "config": cfg, "views": views, "xyz": xyz, "decide": decide, "ring": RING,
    "bytes_per_step": sum(kern_use.values()),
    "bytes_per_step_raw": sum(kern.values()),
    "kernels": short,
    "calibration": cal,
    "per_step": PER_STEP,
    "method": (("every kernel's bytes summed over the launches of %d chained steps (scripts/steps_app.py) / %d; "
                % (PER_STEP, PER_STEP) if PER_STEP else "") + "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over scripts/kbench.py "
               "(one output mode: every k_* kernel launch belongs to the step); " +
               ("HBM bytes per launch = reported bytes x the calibration factor of the kernel's access shapes, "
                "measured on known byte counts by scripts/micro/store_calib in the same call (16-B / 12-B / "
                "3-B / point stores, 8-B / 16-B streaming reads; MI355X_MICROARCH.md HBM: calibrate other "
                "widths on a known byte count); bytes_per_step_raw = 2*FETCH_SIZE + WRITE_SIZE uncorrected"
                if cal else
                "HBM bytes = (2*FETCH_SIZE + WRITE_SIZE) KB * 1024 per launch (gfx950 half-count correction "
                "for wide reads, MI355X_MICROARCH.md HBM; k_cloud's 12-B / 3-B point stores uncalibrated)")),
    "per_kernel_KB": {k: {"FETCH_SIZE": fetch.get(k), "WRITE_SIZE": write.get(k)} for k in kern},
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
