"""Per-kernel SQ / GRBM counter averages from rocprofv3 --pmc CSVs
(counter_collection.csv), several passes merged, kernels matched by a name
substring; prints one table row per (file set, kernel) with derived ratios
(SQ_WAVE_CYCLES split into WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY,
instructions per wave, LDS bank conflicts per LDS-array cycle).

    python scripts/sq_compare.py LABEL=pass1.csv,pass2.csv[,...]:kernel_substring ...
"""
import csv
import sys
from collections import defaultdict


def load(files, sub):
    acc = defaultdict(list)  # counter -> per-dispatch values
    durs = []
    for f in files:
        per = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            d = r["Dispatch_Id"]
            per[d][r["Counter_Name"]] = float(r["Counter_Value"])
            per[d]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for d, cs in per.items():
            for k, v in cs.items():
                if k == "_dur":
                    durs.append(v)
                else:
                    acc[k].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}, (sum(durs) / len(durs) if durs else 0.0), len(durs)


def main():
    for arg in sys.argv[1:]:
        label, rest = arg.split("=", 1)
        files, sub = rest.rsplit(":", 1)
        c, dur, n = load(files.split(","), sub)
        waves = c.get("SQ_WAVES", 1.0)
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        out = {"label": label, "kernel": sub, "dispatches_x_passes": n, "avg_us_profiled": round(dur, 2)}
        for k in sorted(c):
            out[k] = round(c[k], 1)
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in c:
                    out[k + "/WAVE_CYCLES"] = round(c[k] / wc, 3)
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if k in c:
                out[k + "/wave"] = round(c[k] / waves, 1)
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_ACTIVE_INST_LDS"):
            out["LDS_conflict/active_LDS"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_ACTIVE_INST_LDS"], 3)
        if "GRBM_GUI_ACTIVE" in c and dur:
            out["clock_GHz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e3), 3)
        print(out)


if __name__ == "__main__":
    main()
