"""Drop-in for the processing functions of ``multi_point_cloud_process.py``
(the batch GUI) and ``Old/process_cloud.py`` (the CLI).

Same names and signatures as multi_point_cloud_process.py:13-131:
``load_calibration``, ``gray_decode`` (FIXED mask: white > 40 and
white - black > 10, :36-38), ``reconstruct_point_cloud``, ``save_ply``; plus
``process_single`` / ``process_batch``, the per-folder loop of the GUI's
worker thread (:201-257) without Tk.  ``process_batch`` decodes the subfolders
as one multi-view GPU batch when they share a frame size.
"""
from __future__ import annotations

import os

import numpy as np
import scipy.io
import torch

from . import core, io, pipeline, ply
from .sl_system import reconstruct_point_cloud  # identical arithmetic (:73-119)

__all__ = ["load_calibration", "gray_decode", "reconstruct_point_cloud", "save_ply", "process_single",
           "process_batch"]


def load_calibration(calib_path):
    """multi_point_cloud_process.py:13-21 (Old/process_cloud.py:8-23 adds the
    FileNotFoundError, kept here)."""
    if not os.path.exists(calib_path):
        raise FileNotFoundError(f"Calibration file not found at {calib_path}")
    data = scipy.io.loadmat(calib_path)
    return {"Nc": data["Nc"], "Oc": data["Oc"], "wPlaneCol": data["wPlaneCol"], "wPlaneRow": data["wPlaneRow"],
            "cam_K": data["cam_K"]}


def gray_decode(folder, n_cols=1920, n_rows=1080, *, device=None):
    """multi_point_cloud_process.py:23-71 (fixed-threshold mask)."""
    stack, texture, _ = io.read_stack(folder)
    eng = core.engine(device)
    res = eng.decode_triangulate(torch.from_numpy(stack).to(eng.device), n_cols, n_rows, mask_mode="fixed",
                                 maps=True, cloud=False)
    eng.sync()
    return (res["col_map"][0].cpu().numpy(), res["row_map"][0].cpu().numpy(), res["mask"][0].cpu().numpy(),
            texture)


save_ply = ply.save_ply


def process_single(scan_dir, calib_data, *, device=None, log=print):
    """multi_point_cloud_process.py:201-213: decode, reconstruct, save."""
    out_path = os.path.join(scan_dir, os.path.basename(scan_dir) + ".ply")
    log(f"-> Decoding images in {os.path.basename(scan_dir)}...")
    c_map, r_map, mask, texture = gray_decode(scan_dir, device=device)
    log("-> Reconstructing 3D points...")
    points, colors = reconstruct_point_cloud(c_map, r_map, mask, texture, calib_data, device=device)
    log(f"-> Saving {len(points)} points...")
    save_ply(points, colors, out_path)
    return out_path


def process_batch(parent_dir, calib_data, *, n_cols=1920, n_rows=1080, device=None, write=True, log=print,
                  streamed=True, slots=3, keep=True):
    """Batch mode of multi_point_cloud_process.py:241-257: every subfolder with
    images is one view; per-view PLY files are written exactly as the
    reference writes them.  Returns {folder: (P, C)} (empty lists when
    ``keep`` is False: a long scan then holds only ``slots`` views in memory).

    ``streamed`` (default): views of equal frame size and file count go
    through a ``pipeline.ViewPipeline`` -- file decoding of view i+2, H2D of
    view i+1, the kernels of view i and D2H + PLY writing of view i-1 overlap,
    and only the planes the cloud reads are decoded and uploaded.  Otherwise
    all stacks are read first and decoded + triangulated in ONE fused GPU
    launch (merged cloud, per-view offsets)."""
    return process_views(view_folders(parent_dir, log), calib_data, n_cols=n_cols, n_rows=n_rows, device=device,
                         write=write, log=log, streamed=streamed, slots=slots, keep=keep)


def view_folders(parent_dir, log=print) -> list:
    """The batch loop's views (multi_point_cloud_process.py:241-247): sorted
    subfolders that hold images; the others are reported and skipped."""
    subfolders = sorted(f.path for f in os.scandir(parent_dir) if f.is_dir())
    views = [f for f in subfolders if io.list_stack_files(f)]
    for f in subfolders:
        if f not in views:
            log(f"Skipping {os.path.basename(f)} (No images found).")
    return views


def process_views(views, calib_data, *, n_cols=1920, n_rows=1080, device=None, write=True, log=print,
                  streamed=True, slots=3, keep=True):
    """process_batch on a given list of view folders (the shard of one rank in
    a multi-GPU scan, scan360.py).  Returns {folder: (P, C)}."""
    if not views:
        return {}
    if streamed:
        return _process_streamed(views, calib_data, n_cols, n_rows, device, write, log, slots, keep)
    stacks, texes = [], []
    for f in views:
        st, tex, _ = io.read_stack(f)
        stacks.append(st)
        texes.append(tex)
    shapes = {s.shape for s in stacks}
    if len(shapes) != 1:
        raise ValueError(f"batch views differ in stack shape: {sorted(shapes)}")
    eng = core.engine(device)
    H, W = stacks[0].shape[1:]
    eng.set_calibration(calib_data, H, W)
    res = eng.decode_triangulate(torch.from_numpy(np.stack(stacks)).to(eng.device), n_cols, n_rows,
                                 texture=torch.from_numpy(np.stack(texes)).to(eng.device), mask_mode="fixed",
                                 maps=False, cloud=True, xyz_dtype=torch.float64)
    eng.sync()
    cloud = res["cloud"]
    off = cloud.offsets()
    xyz = cloud.xyz[: off[-1]].cpu().numpy()
    bgr = cloud.bgr[: off[-1]].cpu().numpy()
    out = {}
    for v, f in enumerate(views):
        P, C = xyz[off[v]:off[v + 1]], bgr[off[v]:off[v + 1]]
        out[f] = (P, C)
        if write:
            save_ply(P, C, os.path.join(f, os.path.basename(f) + ".ply"))
            log(f"Saved: {os.path.basename(f)}.ply ({len(P)} points)")
    return out


def _process_streamed(views, calib_data, n_cols, n_rows, device, write, log, slots, keep, mask_mode="fixed",
                      raise_errors=False, *, xyz_dtype=torch.float64, poses=None, device_sink=None, host=True,
                      gui_log=False, device_ply=False):
    """Views grouped by (frame size, file count), each group through one
    ``pipeline.ViewPipeline``.  ``raise_errors``: a failing folder raises
    (SLSystem.generate_clouds) instead of being logged and skipped (the batch
    GUI's loop).

    Device-resident use (scan360): ``device_sink(folder, xyz, bgr)`` gets each
    view's points as device tensors (valid during the call), ``poses``
    ({folder: 4x4}) are applied inside k_cloud, and ``host=False`` keeps the
    points in HBM (no D2H, no per-view PLY, nothing in the returned dict).

    ``gui_log`` (SLSystem.generate_clouds): each view's lines are
    generate_cloud's (sl_system.py:574-694: decoding, "Processing N valid
    pixels...", saving, success) instead of the batch GUI's "Saved: ..." line.

    ``device_ply`` (with ``write`` and not ``keep``): each view's PLY is
    formatted on the GPU from the points in HBM (ply.save_ply_device, on the
    pipeline's D2H thread and stream) -- no D2H of the points."""
    files = {f: io.list_stack_files(f) for f in views}
    groups: dict = {}
    for f in views:
        groups.setdefault((io.frame_size(files[f][0]), len(files[f])), []).append(f)
    eng = core.engine(device)
    out = {}
    failed = set()

    def error(f, e):  # the batch loop's per-folder handler (multi_point_cloud_process.py:248-251)
        if raise_errors:
            raise e
        failed.add(f)
        log(f"❌ Error in {os.path.basename(f)}: {e}\n")

    for ((H, W), n_img), group in groups.items():
        try:
            eng.set_calibration(calib_data, H, W)
            pipe = pipeline.ViewPipeline(eng, H=H, W=W, n_img=n_img, n_cols=n_cols, n_rows=n_rows,
                                         mask_mode=mask_mode, xyz_dtype=xyz_dtype, slots=slots,
                                         count_masked=gui_log)
        except (ValueError, IndexError) as e:
            for f in group:
                error(f, e)
            continue

        def fill(i, stack, tex, group=group):
            try:
                # raw BMPs (copy-bound): half the core share, the D2H thread writes the previous
                # views' PLY files meanwhile; PNG / JPEG payloads (decode-bound): the whole share
                fl = files[group[i]]
                share = io.default_workers()
                return io.fill_stack(fl, stack.numpy(), tex.numpy(),
                                     workers=max(1, share // 2) if io.is_raw_bmp(fl[0]) else share)
            except (OSError, ValueError) as e:
                if raise_errors:
                    raise
                error(group[i], e)
                stack[0].zero_()  # white = 0: every pixel masked out, no points
                return True

        def consume(i, xyz, bgr, group=group, pipe=pipe):
            f = group[i]
            if f in failed:
                return
            path = os.path.join(f, os.path.basename(f) + ".ply")
            if gui_log:
                for line in ("Decoding Columns...", "Decoding Rows...", "Reconstructing 3D points...",
                             f"Processing {pipe.masked_count(i)} valid pixels...",
                             f"Saving {len(xyz)} points to {path}..."):
                    log(line)
            if write:
                save_ply(xyz, bgr, path)
                if gui_log:
                    log(f"[Success] Generated {path}")
                else:
                    log(f"Saved: {os.path.basename(f)}.ply ({len(xyz)} points)")
            out[f] = (xyz.copy(), bgr.copy()) if keep else ([], [])

        def on_device(i, xyz, bgr, group=group):
            if group[i] not in failed:
                device_sink(group[i], xyz, bgr)

        def on_device_ply(i, xyz, bgr, group=group, pipe=pipe):
            f = group[i]
            if f in failed:
                return
            path = os.path.join(f, os.path.basename(f) + ".ply")
            if gui_log:
                for line in ("Decoding Columns...", "Decoding Rows...", "Reconstructing 3D points...",
                             f"Processing {pipe.masked_count(i)} valid pixels...",
                             f"Saving {len(xyz)} points to {path}..."):
                    log(line)
            ply.save_ply_device(xyz, bgr, path)
            log(f"[Success] Generated {path}" if gui_log else f"Saved: {os.path.basename(f)}.ply ({len(xyz)} points)")
            out[f] = ([], [])

        gposes = None if poses is None else np.stack([np.asarray(poses[f], np.float64).reshape(4, 4)
                                                      for f in group])
        if device_ply and write and not keep and device_sink is None:
            pipe.run(len(group), fill, None, on_device=on_device_ply, poses=gposes)
            continue
        pipe.run(len(group), fill, consume if host else None,
                 on_device=None if device_sink is None else on_device, poses=gposes)
    return {f: out[f] for f in views if f in out}
