"""Host ingest throughput (file -> uint8 stack in memory) against host cores
(SURVEY.md 8(f)): the capture formats of the reference --
8-bit BMP (sl_system.py:519, the GUI's capture files), JPEG bytes under a .bmp
name (server/server.py:70) and PNG (the glob fallback, :512) -- for one
3840x2160 view, read with io.fill_stack at 1..16 threads.  BMP twice: the raw
reader (io.read_bmp_gray) and Pillow's decoder.  Files are written first, so
reads come from the page cache: this is decode + copy cost, not disk.

    python scripts/ingest_bench.py [--planes 24] [--out profiles/r02_ingest_<host>.jsonl]
"""
import argparse
import json
import os
import platform
import sys
import tempfile
import time

import numpy as np
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structured_light_for_3d_model_replication_amd import io, synth  # noqa: E402


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--planes", type=int, default=24, help="files per view (24 = what the cloud reads)")
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rig = synth.Rig(H=2160, W=3840, Wp=1920, Hp=1080)
    st, _ = synth.render_stack(rig, seed=9, device="cpu")
    st = st.numpy()[: a.planes]
    H, W = st.shape[1:]
    tmp = tempfile.mkdtemp(prefix="ingest_")
    fmts = {}
    for fmt, ext, kw in (("bmp", ".bmp", {}), ("jpeg_as_bmp", ".bmp", {"format": "JPEG", "quality": 95}),
                         ("png", ".png", {})):
        d = os.path.join(tmp, fmt)
        os.makedirs(d)
        for i, p in enumerate(st):
            Image.fromarray(p).save(os.path.join(d, f"{i + 1:02d}{ext}"), **kw)
        fmts[fmt] = io.list_stack_files(d)
    out = np.empty((a.planes, H, W), np.uint8)
    tex = np.empty((H, W, 3), np.uint8)
    lines = []
    host = {"cpu_model": cpu_model(), "host_cores": os.cpu_count(),
            "core_share": int(os.environ.get("OMP_NUM_THREADS", "0")) or None}
    raw_reader = io.read_bmp_gray
    for fmt, files in fmts.items():
        for reader in (("raw", "pillow") if fmt == "bmp" else ("pillow",)):
            io.read_bmp_gray = raw_reader if reader == "raw" else (lambda path, out=None: None)
            for t in [int(x) for x in a.threads.split(",")]:
                io.fill_stack(files, out, tex, workers=t)  # warm (page cache, pool)
                best = float("inf")
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    io.fill_stack(files, out, tex, workers=t)
                    best = min(best, time.perf_counter() - t0)
                ok = bool(np.array_equal(out, st)) if fmt != "jpeg_as_bmp" else None
                rec = {"format": fmt, "reader": reader, "threads": t, "planes": a.planes, "H": H, "W": W,
                       "ms_per_view": 1e3 * best, "Mpx_per_s": a.planes * H * W / best / 1e6,
                       "view_px_per_s": H * W / best, "GB_per_s_decoded": a.planes * H * W / best / 1e9,
                       "bytes_identical": ok, **host}
                lines.append(rec)
                print(json.dumps(rec), flush=True)
    io.read_bmp_gray = raw_reader
    if a.out:
        with open(a.out, "w") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
