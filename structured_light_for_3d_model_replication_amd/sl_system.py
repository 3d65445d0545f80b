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

import numpy as np
import scipy.io
import torch

from . import core, io, ply


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


def decode_and_reconstruct(folder, calib, n_cols=1920, n_rows=1080, *, mask_mode="adaptive", device=None,
                           xyz_dtype=np.float64, count_valid=False):
    """gray_decode + reconstruct_point_cloud fused in one GPU pass (what
    generate_cloud runs).  Row planes are not read: the cloud uses only the
    column code (sl_system.py:624-629).  ``count_valid``: also return the
    number of masked-in pixels (the kernels count them: sl_mask_counts_to)."""
    stack, texture, _ = io.read_stack(folder)
    eng = core.engine(device)
    H, W = stack.shape[1:]
    eng.set_calibration(calib, H, W)
    tdt = torch.float64 if np.dtype(xyz_dtype) == np.float64 else torch.float32
    mc = torch.empty(1, dtype=torch.int64, device=eng.device) if count_valid else None
    res = eng.decode_triangulate(torch.from_numpy(stack).to(eng.device), n_cols, n_rows,
                                 texture=torch.from_numpy(texture).to(eng.device), mask_mode=mask_mode,
                                 maps=False, cloud=True, xyz_dtype=tdt, mask_counts=mc)
    eng.sync()
    cloud = res["cloud"]
    n = cloud.total()
    P, C = cloud.xyz[:n].cpu().numpy().astype(np.float64, copy=False), cloud.bgr[:n].cpu().numpy()
    return (P, C, int(mc.item())) if count_valid else (P, C)


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
        data = scipy.io.loadmat(calib_file)
        if "Oc" not in data:
            raise ValueError("Calibration file missing 'Oc'.")
        calib = _to_numpy_calib(data)
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
        points, colors, n_valid = decode_and_reconstruct(scan_dir, calib, device=self.device, count_valid=True)
        print(f"Processing {n_valid} valid pixels...")
        out_path = os.path.join(scan_dir, os.path.basename(scan_dir) + ".ply")
        print(f"Saving {len(points)} points to {out_path}...")
        ply.save_ply(points, colors, out_path)
        print(f"[Success] Generated {out_path}")

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
                             mask_mode="adaptive", raise_errors=True, gui_log=True)
        return [os.path.join(d, os.path.basename(d) + ".ply") for d in scan_dirs]
