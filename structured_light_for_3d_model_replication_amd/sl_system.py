"""Drop-in for the reconstruction half of ``server/sl_system.py``.

``SLSystem.generate_cloud(scan_dir, calib_file)`` keeps the reference's name,
signature, prints, exceptions and output file (sl_system.py:483-694); the two
functions it nests are exposed here at module level with the reference's
signatures:

* ``gray_decode(folder, n_cols=1920, n_rows=1080)`` -> (col_map int32,
  row_map int32, valid_mask bool, texture uint8 BGR)   (sl_system.py:508-580)
* ``reconstruct_point_cloud(col_map, row_map, mask, texture, calib)`` ->
  (P float64 (N,3), C uint8 (N,3) BGR)                 (sl_system.py:584-653)

The arithmetic runs in libslgpu.so on the GPU (no CPU fallback).  Points are
returned bit-identical to the reference (the kernels compute in f64 in the
reference's operation order and the f64 output mode is used here).

Only the reconstruction path is provided; projector / capture / calibration
methods of the reference class are outside this package's scope.
"""
from __future__ import annotations

import os
import threading

import numpy as np
import scipy.io
import torch

from . import core, io, pipeline, ply


def _to_numpy_calib(data) -> dict:
    # the same keys (and KeyError on a missing one) as sl_system.py:498-504
    return {k: data[k] for k in ("Nc", "Oc", "wPlaneCol", "wPlaneRow", "cam_K")}


def gray_decode(folder, n_cols=1920, n_rows=1080, *, mask_mode="adaptive", device=None):
    """gray_decode of sl_system.py:508-580 (adaptive shadow/contrast mask)."""
    stack, texture, _ = io.read_stack(folder)
    eng = core.engine(device)
    st = torch.from_numpy(stack).to(eng.device)
    print("Decoding Columns...")
    print("Decoding Rows...")
    res = eng.decode_triangulate(st, n_cols, n_rows, mask_mode=mask_mode, maps=True, cloud=False)
    eng.sync()
    return (res["col_map"][0].cpu().numpy(), res["row_map"][0].cpu().numpy(), res["mask"][0].cpu().numpy(),
            texture)


def reconstruct_point_cloud(col_map, row_map, mask, texture, calib, *, device=None, xyz_dtype=np.float64):
    """reconstruct_point_cloud of sl_system.py:584-653.  ``row_map`` is unused,
    as in the reference."""
    del row_map
    print("Reconstructing 3D points...")
    col_map = np.asarray(col_map)
    h, w = col_map.shape
    eng = core.engine(device)
    eng.set_calibration(calib, h, w)
    mask = np.asarray(mask)
    print(f"Processing {int(np.count_nonzero(mask))} valid pixels...")
    tdt = torch.float64 if np.dtype(xyz_dtype) == np.float64 else torch.float32
    cloud = eng.triangulate_maps(torch.from_numpy(np.ascontiguousarray(col_map, dtype=np.int32)),
                                 torch.from_numpy(np.ascontiguousarray(mask != 0)),
                                 torch.from_numpy(np.ascontiguousarray(np.asarray(texture).reshape(h, w, 3),
                                                                       dtype=np.uint8)),
                                 xyz_dtype=tdt)
    eng.sync()
    n = cloud.total()
    return cloud.xyz[:n].cpu().numpy().astype(np.float64, copy=False), cloud.bgr[:n].cpu().numpy()


_STAGE = {}  # (device, n_up, H, W) -> the one-view path's pinned host and device stack / texture buffers
_STAGE_LOCK = threading.Lock()


def _stage(dev, n_up, H, W):
    key = (str(dev), n_up, H, W)
    if key not in _STAGE:
        if len(_STAGE) >= 2:  # a frame-size change releases the older buffers
            _STAGE.pop(next(iter(_STAGE)))
        _STAGE[key] = (torch.empty((n_up, H, W), dtype=torch.uint8, pin_memory=True),
                       torch.empty((H, W, 3), dtype=torch.uint8, pin_memory=True),
                       torch.empty((n_up, H, W), dtype=torch.uint8, device=dev),
                       torch.empty((H, W, 3), dtype=torch.uint8, device=dev))
    return _STAGE[key]


def _decode_device(folder, calib, n_cols, n_rows, mask_mode, device, xyz_dtype, count_valid, prepared):
    """decode_and_reconstruct's work, the cloud left on the device -> (xyz,
    bgr device tensors of the n points, masked-in pixel count or None)."""
    files = io.list_stack_files(folder)
    n_up = pipeline.planes_for_cloud(len(files), n_cols, n_rows)
    H, W = io.frame_size(files[0])
    eng = core.engine(device)
    eng.set_calibration(calib, H, W, _prepared=prepared)
    tdt = torch.float64 if np.dtype(xyz_dtype) == np.float64 else torch.float32
    mc = torch.empty(1, dtype=torch.int64, device=eng.device) if count_valid else None
    with _STAGE_LOCK:  # the staging buffers are shared by the calls of this process
        hs, ht, ds, dt = _stage(eng.device, n_up, H, W)
        s = torch.cuda.current_stream(eng.device)

        def upload(j):  # each plane's H2D starts on the decoding thread as soon as the plane is in place
            with torch.cuda.stream(s):
                ds[j].copy_(hs[j], non_blocking=True)
        gray_tex = io.fill_stack(files, hs.numpy(), ht.numpy(), on_plane=upload)
        if not gray_tex:
            dt.copy_(ht, non_blocking=True)
        res = eng.decode_triangulate(ds, n_cols, n_rows, texture=None if gray_tex else dt, mask_mode=mask_mode,
                                     maps=False, cloud=True, xyz_dtype=tdt, mask_counts=mc, stream=s)
        eng.sync(s)
    cloud = res["cloud"]
    n = cloud.total()
    return cloud.xyz[:n], cloud.bgr[:n], (int(mc.item()) if count_valid else None)


def decode_and_reconstruct(folder, calib, n_cols=1920, n_rows=1080, *, mask_mode="adaptive", device=None,
                           xyz_dtype=np.float64, count_valid=False, prepared=None):
    """gray_decode + reconstruct_point_cloud fused in one GPU pass (what
    generate_cloud runs).  The whole file list is checked with gray_decode's
    rules (sl_system.py:515-516, 549-554: ValueError below 4 files,
    IndexError for a pattern without its inverse), but only the files the
    cloud reads are decoded -- white, black and the column pairs (24 of 46 for
    11 + 11 bits): reconstruct_point_cloud uses only col_map (:624-629) -- into
    pinned buffers kept for the next call, each plane uploaded from there
    as soon as it is decoded (the uploads overlap the remaining decodes).
    ``count_valid``: also return the number of masked-in pixels (the kernels
    count them: sl_mask_counts_to).  ``prepared``: calibration_key(calib, H,
    W) when the caller has it (SLSystem.generate_cloud caches it per file)."""
    xyz, bgr, n_valid = _decode_device(folder, calib, n_cols, n_rows, mask_mode, device, xyz_dtype, count_valid,
                                       prepared)
    P, C = xyz.cpu().numpy().astype(np.float64, copy=False), bgr.cpu().numpy()
    return (P, C, n_valid) if count_valid else (P, C)


def index_error_stage(n_files: int, n_cols: int = 1920, n_rows: int = 1080):
    """Where gray_decode's decode_sequence (sl_system.py:544-577) reads past
    the last file -- the IndexError of its ``files[current_idx]`` (:553-554)
    -- while decoding the columns ("cols"), the rows ("rows"), or never
    (None); a short stack that simply runs out of files is not an error
    (:550)."""
    idx = 2
    for stage, n in (("cols", n_cols), ("rows", n_rows)):
        for _ in range(int(np.ceil(np.log2(n)))):
            if idx >= n_files:
                break
            if idx + 1 >= n_files:
                return stage
            idx += 2
    return None


_CALIB = {}  # calib file identity -> (calib dict, {(H, W): calibration_key}); see SLSystem._calib
_CALIB_LOCK = threading.Lock()


class SLSystem:
    """Reconstruction part of server/sl_system.py:14 ``SLSystem``."""

    def __init__(self, device=None):
        self.window_name = "Projector"
        self.device = device

    def generate_cloud(self, scan_dir, calib_file):
        """sl_system.py:483-694: decode ``scan_dir`` with ``calib_file`` and write
        ``<scan_dir>/<basename>.ply``."""
        if not os.path.exists(calib_file):
            raise FileNotFoundError(f"Calibration file not found at {calib_file}")
        print(f"[Process] Processing {scan_dir} using {calib_file}...")
        calib, keys = self._calib(calib_file)
        # gray_decode's checks and prints, in the reference's order (:510-516,
        # :549-554, :574-577): the stack's faults raise where it would
        n_files = len(io.list_stack_files(scan_dir))
        if n_files < 4:
            raise ValueError("Not enough images in folder to decode.")
        stage = index_error_stage(n_files)
        print("Decoding Columns...")
        if stage == "cols":
            raise IndexError("list index out of range")
        print("Decoding Rows...")
        if stage == "rows":
            raise IndexError("list index out of range")
        print("Reconstructing 3D points...")
        files = io.list_stack_files(scan_dir)
        hw = io.frame_size(files[0])
        with _CALIB_LOCK:
            if hw not in keys:  # the content key (and pinhole check) of this calibration at this frame size
                keys[hw] = core.Reconstructor.calibration_key(calib, *hw)
            prepared = keys[hw]
        xyz, bgr, n_valid = _decode_device(scan_dir, calib, 1920, 1080, "adaptive", self.device, np.float64, True,
                                           prepared)
        print(f"Processing {n_valid} valid pixels...")
        out_path = os.path.join(scan_dir, os.path.basename(scan_dir) + ".ply")
        print(f"Saving {xyz.shape[0]} points to {out_path}...")
        # the text formatted on the GPU from the f64 points in HBM (the same
        # bytes as ply.save_ply: one digit code), no D2H of the points
        ply.save_ply_device(xyz, bgr, out_path)
        print(f"[Success] Generated {out_path}")

    @staticmethod
    def _calib(calib_file):
        """calib.mat loaded as generate_cloud loads it (sl_system.py:496-504:
        scipy.io.loadmat, the 'Oc' check, the five arrays), kept while the
        file is the same (path, inode, size, mtime): a GUI session decodes
        many scans with one calibration, and a 4K calib.mat's Nc table takes
        ~0.2 s to load and as long again to key."""
        st = os.stat(calib_file)
        ident = (os.path.realpath(calib_file), st.st_ino, st.st_size, st.st_mtime_ns)
        with _CALIB_LOCK:
            hit = _CALIB.get(ident)
        if hit is not None:
            return hit
        data = scipy.io.loadmat(calib_file)
        if "Oc" not in data:
            raise ValueError("Calibration file missing 'Oc'.")
        hit = (_to_numpy_calib(data), {})
        with _CALIB_LOCK:
            for k in [k for k in _CALIB if k[0] == ident[0]]:
                del _CALIB[k]  # an older version of this file
            _CALIB[ident] = hit
        return hit

    def generate_clouds(self, scan_dirs, calib_file, *, slots=3):
        """Batched ``generate_cloud``: every folder of ``scan_dirs``
        gets the ``<scan_dir>/<basename>.ply`` that generate_cloud writes for
        it, byte for byte (adaptive mask, f64 points, sl_system.py:483-694).
        Views stream through one ``pipeline.ViewPipeline`` per frame size: file
        decoding, H2D, the kernels and D2H + PLY writing of neighbouring views
        overlap.  The calibration checks and exceptions are generate_cloud's;
        a folder with fewer than 4 images raises its ValueError before any
        view is processed.  Each view then prints generate_cloud's lines
        ("Decoding Columns..." ... "Processing N valid pixels..." ... "[Success]
        Generated ...") as its cloud is written.  Returns the PLY paths in
        ``scan_dirs`` order."""
        from . import multi_point_cloud_process as mp
        if not os.path.exists(calib_file):
            raise FileNotFoundError(f"Calibration file not found at {calib_file}")
        data = scipy.io.loadmat(calib_file)
        if "Oc" not in data:
            raise ValueError("Calibration file missing 'Oc'.")
        calib = _to_numpy_calib(data)
        scan_dirs = [str(d) for d in scan_dirs]
        for d in scan_dirs:
            print(f"[Process] Processing {d} using {calib_file}...")
            if len(io.list_stack_files(d)) < 4:  # sl_system.py:515-516
                raise ValueError("Not enough images in folder to decode.")
        mp._process_streamed(scan_dirs, calib, 1920, 1080, self.device, True, print, slots, False,
                             mask_mode="adaptive", raise_errors=True, gui_log=True, device_ply=True)
        return [os.path.join(d, os.path.basename(d) + ".ply") for d in scan_dirs]
