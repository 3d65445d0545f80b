"""User-visible end-to-end rate at HEAD: scan folders on disk ->
PLY files on disk, the way the GUI and the batch GUI run them.

    python scripts/e2e_bench.py [--views 6] [--formats bmp,png,jpg] [--H 2160 --W 3840]

For each capture format, ``views`` 4K scan folders of 46 files (config-2 rig,
11 + 11 bits with inverses) are written to $TMPDIR:
  bmp   8-bit single-channel BMP (what sl_system.py:519 reads back)
  png   8-bit single-channel PNG (the *.png fallback, sl_system.py:512-513)
  jpg   colour JPEG bytes saved under .bmp names (server/server.py:70: the
        Android capture's upload is written as-is)
Legs (one JSON line each):
  gui_stages  generate_cloud's work for one folder at a time, stage by stage
              (median over the folders), as sl_system.decode_and_reconstruct
              runs it: file decoding (the 24 files the cloud reads into pinned
              staging buffers, io.fill_stack, 8 threads), H2D, the kernels
              (k_stats, k_decode, k_cloud; f64 xyz, generate_cloud's mode), D2H
              of the points, the ASCII PLY (sl_system.py:665-691: native
              formatter, 16 threads) -- and SLSystem.generate_cloud's own wall
              time for the same folders (stdout suppressed; the calib.mat holds
              a full 3 x H*W Nc table, as calibrate_final writes it: the first
              call loads and keys it, later ones reuse it)
  batch       SLSystem.generate_clouds over all folders (pipeline.ViewPipeline:
              24 cloud planes decoded into pinned slots, H2D, kernels, D2H and
              the PLY of neighbouring views overlapped): views/s, and the
              pipeline's host-side totals
Disk: one format's folders at a time (~2.5 GB for 6 BMP views + their PLYs).
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes
import io as _io
import json
import os
import shutil
import statistics
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import scipy.io
import torch
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structured_light_for_3d_model_replication_amd import _lib, core, io, pipeline, ply, sl_system, synth  # noqa: E402


def write_folder(folder, stack, fmt, pool):
    os.makedirs(folder)

    def one(j):
        a = stack[j]
        if fmt == "png":
            Image.fromarray(a).save(os.path.join(folder, f"{j + 1:02d}.png"))
        elif fmt == "jpg":  # colour JPEG bytes under a .bmp name (server.py:70)
            with open(os.path.join(folder, f"{j + 1:02d}.bmp"), "wb") as f:
                Image.fromarray(np.repeat(a[:, :, None], 3, axis=2)).save(f, format="JPEG", quality=95)
        else:
            Image.fromarray(a).save(os.path.join(folder, f"{j + 1:02d}.bmp"))
    list(pool.map(one, range(len(stack))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=6)
    ap.add_argument("--formats", default="bmp,png,jpg")
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--W", type=int, default=3840)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rig = synth.Rig(H=a.H, W=a.W)
    cal = synth.make_calibration(rig, with_Nc=True)
    stacks = []
    for v in range(min(a.views, 4)):  # 4 distinct synthetic views, cycled
        s, _ = synth.render_stack(rig, seed=3000 + v, view_deg=10.0 * v, device="cpu")
        stacks.append(s.numpy())
    root = tempfile.mkdtemp(prefix="sl_e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
    calib_file = os.path.join(root, "calib.mat")
    scipy.io.savemat(calib_file, {k: np.asarray(v) for k, v in cal.items()})
    eng = core.engine(dev)
    pool = ThreadPoolExecutor(16)
    slsys = sl_system.SLSystem()
    px = a.H * a.W
    try:
        for fmt in a.formats.split(","):
            fdir = os.path.join(root, fmt)
            os.makedirs(fdir)
            t0 = time.perf_counter()
            folders = []
            for v in range(a.views):
                f = os.path.join(fdir, f"scan_{v:03d}")
                write_folder(f, stacks[v % len(stacks)], fmt, pool)
                folders.append(f)
            write_s = time.perf_counter() - t0
            disk = sum(os.path.getsize(os.path.join(folders[0], x)) for x in os.listdir(folders[0]))
            # page cache warm for every leg (the files were just written)
            # ---- gui_stages: generate_cloud's work, stage by stage ----
            st = {k: [] for k in ("decode_files", "h2d", "kernels", "ply")}
            host_ply = {k: [] for k in ("d2h", "ply_host", "format_only")}
            pts = []
            eng.set_calibration(cal, a.H, a.W)
            for f in folders:
                t0 = time.perf_counter()
                files = io.list_stack_files(f)
                n_up = pipeline.planes_for_cloud(len(files))
                hs, ht, ds, dt = sl_system._stage(dev, n_up, *io.frame_size(files[0]))
                gray = io.fill_stack(files, hs.numpy(), ht.numpy())
                t1 = time.perf_counter()
                ds.copy_(hs, non_blocking=True)
                if not gray:
                    dt.copy_(ht, non_blocking=True)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                res = eng.decode_triangulate(ds, texture=None if gray else dt, maps=False, cloud=True,
                                             xyz_dtype=torch.float64)
                eng.sync()
                t3 = time.perf_counter()
                cl = res["cloud"]
                n = cl.total()
                path = os.path.join(f, os.path.basename(f) + ".ply")
                ply.save_ply_device(cl.xyz[:n], cl.bgr[:n], path)  # generate_cloud's PLY: formatted on the GPU
                t4 = time.perf_counter()
                for k, (x, y) in zip(st, ((t0, t1), (t1, t2), (t2, t3), (t3, t4))):
                    st[k].append(1e3 * (y - x))
                # beside it, the host formatter's route: D2H of the points, format + write on 16 threads
                os.remove(path)
                t5 = time.perf_counter()
                P, C = cl.xyz[:n].cpu().numpy(), cl.bgr[:n].cpu().numpy()
                t6 = time.perf_counter()
                ply.save_ply(P, C, path)
                t7 = time.perf_counter()
                ln = ctypes.c_int64()  # the formatting alone (sl_format_ply's size query formats every line)
                _lib.check(_lib.load().sl_format_ply(P.ctypes.data, _lib.SL_XYZ_F64, C.ctypes.data, len(P), ply._THREADS,
                                                     None, 0, ctypes.byref(ln)), None, "sl_format_ply")
                t8 = time.perf_counter()
                for k, (x, y) in zip(host_ply, ((t5, t6), (t6, t7), (t7, t8))):
                    host_ply[k].append(1e3 * (y - x))
                pts.append(n)
                del res, cl, P, C
            ply_bytes = os.path.getsize(os.path.join(folders[-1], os.path.basename(folders[-1]) + ".ply"))
            gc_ms = []
            for f in folders:
                # a new scan's folder: generate_cloud writes a new file (overwriting a 250 MB PLY
                # that sits in the page cache costs ~40 ms more: the old pages are freed first)
                os.remove(os.path.join(f, os.path.basename(f) + ".ply"))
                t0 = time.perf_counter()
                with contextlib.redirect_stdout(_io.StringIO()):
                    slsys.generate_cloud(f, calib_file)
                gc_ms.append(1e3 * (time.perf_counter() - t0))
            rerun_ms = []
            for f in folders:
                # a re-run over the same folders: each PLY is there already (the writer renames it
                # away and unlinks it beside the write instead of truncating it in its path)
                t0 = time.perf_counter()
                with contextlib.redirect_stdout(_io.StringIO()):
                    slsys.generate_cloud(f, calib_file)
                rerun_ms.append(1e3 * (time.perf_counter() - t0))
            time.sleep(0.5)  # (the replaced files' unlinks)
            # where generate_cloud's wall time goes beyond the stages: one call under cProfile
            import cProfile
            import pstats
            prof = cProfile.Profile()
            os.remove(os.path.join(folders[0], os.path.basename(folders[0]) + ".ply"))
            with contextlib.redirect_stdout(_io.StringIO()):
                prof.enable()
                slsys.generate_cloud(folders[0], calib_file)
                prof.disable()
            ps = pstats.Stats(prof)
            top = sorted(((v[3], f"{os.path.basename(k[0])}:{k[1]}:{k[2]}") for k, v in ps.stats.items()),
                         reverse=True)[:18]
            profile_top = [[round(1e3 * t, 2), name] for t, name in top]
            med = {k: statistics.median(v) for k, v in st.items()}
            limiting = max(med, key=med.get)
            print(json.dumps({"leg": "gui_stages", "format": fmt, "views": a.views, "H": a.H, "W": a.W,
                              "files_per_view": 46, "bytes_on_disk_per_view": disk,
                              "stage_ms_median": med, "stage_ms_all": st, "limiting_stage": limiting,
                              "host_ply_route_ms_median": {k: statistics.median(v) for k, v in host_ply.items()},
                              "sum_of_stages_ms": sum(med.values()),
                              "generate_cloud_ms_median": statistics.median(gc_ms), "generate_cloud_ms": gc_ms,
                              "generate_cloud_rerun_ms_median": statistics.median(rerun_ms),
                              "generate_cloud_rerun_ms": rerun_ms,
                              "views_per_s_gui": 1e3 / statistics.median(gc_ms),
                              "points_per_view": int(statistics.median(pts)), "ply_bytes_per_view": ply_bytes,
                              "folders_write_s": write_s, "generate_cloud_profile_cum_ms": profile_top,
                              "note": "page cache warm; decode_files = the 24 cloud files into pinned staging "
                                      "(io.fill_stack, 8 threads; the colour re-read of file 0 when it is not "
                                      "single-channel); kernels = decode_triangulate + sync (f64 xyz); ply = the "
                                      "text formatted on the GPU, copied back in chunks, written (generate_cloud's "
                                      "route); host_ply_route = D2H of the points + the host formatter on 16 "
                                      "threads (+ its formatting alone); generate_cloud_ms[0] includes the "
                                      "calib.mat load + key (a 3 x H*W Nc table)"}), flush=True)
            # ---- batch: generate_clouds, pipelined ----
            for f in folders:
                os.remove(os.path.join(f, os.path.basename(f) + ".ply"))
            with contextlib.redirect_stdout(_io.StringIO()):
                slsys.generate_clouds(folders[:2], calib_file)  # warm: pools, pinned slots
            for f in folders[:2]:  # the timed run writes new files, as the GUI legs do (no overwrite cost)
                os.remove(os.path.join(f, os.path.basename(f) + ".ply"))
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(_io.StringIO()):
                slsys.generate_clouds(folders, calib_file)
            el = time.perf_counter() - t0
            # the pipeline's stages in isolation, per view: 24 planes decoded into one buffer, the PLY
            files = io.list_stack_files(folders[0])
            buf = np.empty((24, a.H, a.W), np.uint8)
            tex = np.empty((a.H, a.W, 3), np.uint8)
            fills = []
            for f in folders:
                t1 = time.perf_counter()
                io.fill_stack(io.list_stack_files(f), buf, tex)
                fills.append(1e3 * (time.perf_counter() - t1))
            print(json.dumps({"leg": "batch", "format": fmt, "views": a.views, "wall_s": el,
                              "views_per_s": a.views / el, "px_per_s": a.views * px / el,
                              "fill_24_planes_ms_median": statistics.median(fills),
                              "ply_ms_median": med["ply"], "kernels_ms_median": med["kernels"],
                              "limiting_stage": "decode_files" if statistics.median(fills) > med["ply"] else "ply",
                              "note": "SLSystem.generate_clouds (ViewPipeline, 3 slots: decode of the 24 cloud "
                                      "planes, H2D, kernels, D2H, PLY overlapped); stage costs in isolation beside"}),
                  flush=True)
            shutil.rmtree(fdir, ignore_errors=True)
            del files
    finally:
        shutil.rmtree(root, ignore_errors=True)
        pool.shutdown()


if __name__ == "__main__":
    main()
