"""Load the golden fixtures written by tests/golden/make_golden.py."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    d["calib"] = {k[len("calib_"):]: v for k, v in d.items() if k.startswith("calib_")}
    return d


def names(func=None):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        n = os.path.splitext(os.path.basename(p))[0]
        if func is None or load(n)["meta"].get("func") in func:
            out.append(n)
    return out


def ply_text(name):
    with open(os.path.join(GOLDEN, name), encoding="utf-8") as f:
        return f.read()
