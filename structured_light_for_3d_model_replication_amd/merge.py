"""Merge stage on the GPU (server/processing.py:116-182).

``merge_pro_360`` concatenates the per-view clouds in a common frame, then
``voxel_down_sample`` (:171) and ``remove_statistical_outlier(20, 2.0)`` +
``select_by_index`` (:174-175), and writes the result.  These are Open3D calls in
the reference.  Here they are HIP kernels of libslgpu.so (csrc/slmerge.hip)
with Open3D's arithmetic: same voxel grid, sums in point order, exact kNN, and
sequential cloud statistics.  Voxel output is in ascending voxel key rather than
Open3D's hash order.

Then ``estimate_normals(KDTreeSearchParamHybrid(radius=2 voxel, max_nn=30))``
(:178) and ``write_point_cloud`` (:181).  Open3D is not in this image, so
parity is unpinned; oracle/merge_oracle.py is the restatement the tests check
against.

The reference aligns the views by FPFH + RANSAC + ICP (:145-157).  That
registration is out of scope.  ``merge_pro_360_posed`` takes the poses instead:
the turntable's known poses, or the same ones ``Reconstructor.decode_triangulate``
applies inside k_cloud.
"""
from __future__ import annotations

import ctypes
import glob
import os
import re
import threading

import numpy as np
import torch

from . import _lib, core, ply

_engines: dict = {}
_engines_lock = threading.Lock()


def _engine(device) -> core.Reconstructor:
    dev = torch.device(device if device is not None else "cuda")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    with _engines_lock:
        if idx not in _engines:
            _engines[idx] = core.Reconstructor(torch.device("cuda", idx))
        return _engines[idx]


def _f64(points, dev) -> torch.Tensor:
    P = torch.as_tensor(points)
    if P.dim() != 2 or P.shape[1] != 3:
        raise ValueError("points must be (N, 3)")
    return P.to(device=dev, dtype=torch.float64).contiguous()


def _u8(colors, dev, n) -> torch.Tensor | None:
    if colors is None:
        return None
    C = torch.as_tensor(colors).to(device=dev, dtype=torch.uint8).contiguous()
    if C.shape != (n, 3):
        raise ValueError("colors must be (N, 3) uint8")
    return C


def _ptr(t):
    return None if t is None else t.data_ptr()


def voxel_down_sample(points, colors=None, voxel_size: float = 0.02, *, device=None):
    """PointCloud.voxel_down_sample -> (points f64 [M,3], colors u8 [M,3] | None) on the device."""
    eng = _engine(device)
    P = _f64(points, eng.device)
    n = P.shape[0]
    C = _u8(colors, eng.device, n)
    out = torch.empty((max(n, 1), 3), dtype=torch.float64, device=eng.device)
    oc = None if C is None else torch.empty((max(n, 1), 3), dtype=torch.uint8, device=eng.device)
    m = ctypes.c_int64()
    with eng._lock:
        _lib.check(eng._L.sl_voxel_downsample(eng._ctx, _ptr(P), _ptr(C), n, float(voxel_size), out.data_ptr(),
                                              _ptr(oc), ctypes.byref(m), eng._stream(None)),
                   eng._ctx, "sl_voxel_downsample")
    k = m.value
    return out[:k], (None if oc is None else oc[:k])


def remove_statistical_outlier(points, nb_neighbors: int = 20, std_ratio: float = 2.0, *, device=None):
    """PointCloud.remove_statistical_outlier -> (ind int64 [K] ascending, mean kNN distance f64 [N])."""
    eng = _engine(device)
    P = _f64(points, eng.device)
    n = P.shape[0]
    avg = torch.empty(max(n, 1), dtype=torch.float64, device=eng.device)
    ind = torch.empty(max(n, 1), dtype=torch.int64, device=eng.device)
    k = ctypes.c_int64()
    with eng._lock:
        _lib.check(eng._L.sl_statistical_outliers(eng._ctx, _ptr(P), n, int(nb_neighbors), float(std_ratio),
                                                  avg.data_ptr(), ind.data_ptr(), ctypes.byref(k),
                                                  eng._stream(None)),
                   eng._ctx, "sl_statistical_outliers")
    return ind[: k.value], avg[:n]


def select_by_index(points, colors, ind, *, device=None):
    """PointCloud.select_by_index -> (points, colors | None) on the device."""
    eng = _engine(device)
    P = _f64(points, eng.device)
    C = _u8(colors, eng.device, P.shape[0])
    I = torch.as_tensor(ind).to(device=eng.device, dtype=torch.int64).contiguous()
    m = I.shape[0]
    if m and (int(I.min()) < 0 or int(I.max()) >= P.shape[0]):
        raise IndexError("index out of range")
    out = torch.empty((max(m, 1), 3), dtype=torch.float64, device=eng.device)
    oc = None if C is None else torch.empty((max(m, 1), 3), dtype=torch.uint8, device=eng.device)
    with eng._lock:
        _lib.check(eng._L.sl_select_by_index(eng._ctx, _ptr(P), _ptr(C), I.data_ptr(), m, out.data_ptr(), _ptr(oc),
                                             eng._stream(None)), eng._ctx, "sl_select_by_index")
    return out[:m], (None if oc is None else oc[:m])


def transform(points, pose, *, device=None) -> torch.Tensor:
    """PointCloud.transform(pose) on a device copy of points (row order ((m0 x + m1 y) + m2 z) + m3)."""
    eng = _engine(device)
    P = _f64(points, eng.device).clone()
    M = torch.as_tensor(np.asarray(pose, dtype=np.float64).reshape(16)).to(eng.device)
    with eng._lock:
        _lib.check(eng._L.sl_transform_points(eng._ctx, P.data_ptr(), P.shape[0], M.data_ptr(), eng._stream(None)),
                   eng._ctx, "sl_transform_points")
    return P


def estimate_normals(points, radius: float, max_nn: int = 30, *, device=None) -> torch.Tensor:
    """PointCloud.estimate_normals(KDTreeSearchParamHybrid(radius, max_nn)) of a
    cloud without normals (processing.py:178) -> normals f64 [N,3] on the
    device (sl_estimate_normals; max_nn <= 32)."""
    eng = _engine(device)
    P = _f64(points, eng.device)
    n = P.shape[0]
    out = torch.empty((max(n, 1), 3), dtype=torch.float64, device=eng.device)
    with eng._lock:
        _lib.check(eng._L.sl_estimate_normals(eng._ctx, _ptr(P), n, float(radius), int(max_nn), out.data_ptr(),
                                              eng._stream(None)), eng._ctx, "sl_estimate_normals")
    return out[:n]


def pool_trim(device=None) -> int:
    """Release the merge kernels' pooled scratch buffers of ``device``
    (sl_merge_pool_trim); returns the bytes released."""
    eng = _engine(device)
    out = ctypes.c_int64()
    _lib.check(eng._L.sl_merge_pool_trim(eng.device.index, ctypes.byref(out)), None, "sl_merge_pool_trim")
    return out.value


def postprocess(points, colors, voxel_size: float, nb_neighbors: int = 20, std_ratio: float = 2.0, *,
                device=None):
    """processing.py:171-175: voxel_down_sample, then remove_statistical_outlier + select_by_index."""
    P, C = voxel_down_sample(points, colors, voxel_size, device=device)
    ind, _ = remove_statistical_outlier(P, nb_neighbors, std_ratio, device=device)
    return select_by_index(P, C, ind, device=device)


def ply_files(folder, order: str = "lexicographic") -> list:
    """The clouds a 360 merge reads, in its order: ``"lexicographic"`` is
    processing.py:121's ``sorted(glob('*.ply'))`` (``view_100deg`` before
    ``view_10deg``); ``"numeric"`` is Old/new360Merge.py:7-20's key, the first
    integer in the file name (0 when none; ties keep name order)."""
    if order == "lexicographic":
        return sorted(glob.glob(os.path.join(folder, "*.ply")))
    if order == "numeric":
        names = sorted(f for f in os.listdir(folder) if f.lower().endswith(".ply"))

        def first_int(name):
            m = re.search(r"\d+", name)
            return int(m.group()) if m else 0
        return [os.path.join(folder, f) for f in sorted(names, key=first_int)]
    raise ValueError("order must be 'lexicographic' or 'numeric'")


def merge_pro_360_posed(input_folder, output_path, poses, voxel_size: float = 0.02, *, device=None,
                        binary: bool = True, order: str = "lexicographic"):
    """merge_pro_360 (processing.py:116-182) with known per-file poses instead
    of the FPFH/RANSAC/ICP estimate: files in ``ply_files(order)`` order
    (default: the reference's lexicographic one), file i moved by ``poses[i]``
    (4x4), merged, post-processed, normals estimated (radius 2 voxel, max_nn 30,
    :178) and written as o3d.io.write_point_cloud writes it (binary, double
    xyz + normals, uchar RGB: ply.save_ply_open3d; ``binary=False``: the same
    properties in ASCII).  Returns (points, colors, normals) on the device."""
    print(f"[Merge 360] Loading clouds from {input_folder}...")
    files = ply_files(input_folder, order)
    if len(files) < 2:
        raise ValueError("Need at least 2 .ply files to merge.")
    poses = np.asarray(poses, dtype=np.float64).reshape(-1, 4, 4)
    if len(poses) != len(files):
        raise ValueError(f"{len(files)} clouds but {len(poses)} poses")
    eng = _engine(device)
    parts_p, parts_c = [], []
    for f, M in zip(files, poses):
        P, C = ply.read_ply(f)
        parts_p.append(transform(P, M, device=eng.device))
        parts_c.append(torch.from_numpy(C).to(eng.device))
    print(f"[Merge 360] Loaded {len(files)} clouds. Applying the given poses...")
    merged_p = torch.cat(parts_p)
    merged_c = torch.cat(parts_c)
    print("[Merge 360] Post-processing (Downsample + Outlier removal)...")
    P, C = postprocess(merged_p, merged_c, voxel_size, device=eng.device)
    N = estimate_normals(P, voxel_size * 2, 30, device=eng.device)
    ply.save_ply_open3d(P.cpu().numpy(), C.cpu().numpy(), output_path, normals=N.cpu().numpy(), binary=binary)
    print(f"[Merge 360] Saved merged cloud to {output_path}")
    return P, C, N
