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

Registration.  The reference aligns consecutive views by FPFH + RANSAC
(a global estimate) refined by point-to-plane ICP (:145-157) and accumulates
the transforms (:159-167).  ``merge_pro_360`` keeps that flow on the GPU:
``compute_fpfh_feature`` (sl_compute_fpfh), ``registration_ransac_based_on_
feature_matching`` (sl_ransac_feature_matching) and ``registration_icp``
(sl_icp_point_to_plane) -- Open3D's algorithms; parity vs Open3D unpinned,
oracle/registration_oracle.py and oracle/merge_oracle.py restate them.  With
``seed_poses`` (a turntable's known poses) the RANSAC estimate is replaced by
the relative pose between the two views.
``merge_pro_360_posed`` skips registration and takes the poses as they are
(the same ones ``Reconstructor.decode_triangulate`` applies inside k_cloud).
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


def registration_icp(source, target, target_normals, max_correspondence_distance: float, init=None, *,
                     max_iteration: int = 30, relative_fitness: float = 1e-6, relative_rmse: float = 1e-6,
                     device=None) -> dict:
    """o3d.pipelines.registration.registration_icp(source, target,
    max_correspondence_distance, init, TransformationEstimationPointToPlane(),
    ICPConvergenceCriteria(relative_fitness, relative_rmse, max_iteration))
    (processing.py:154-156) on the GPU -> {"transformation": 4x4 numpy,
    "fitness", "inlier_rmse", "iterations"}.  ``target_normals``: the target's
    normals (estimate_normals, as merge_pro_360 computes them)."""
    eng = _engine(device)
    S = _f64(source, eng.device)
    T = _f64(target, eng.device)
    N = _f64(target_normals, eng.device)
    if N.shape != T.shape:
        raise ValueError("TransformationEstimationPointToPlane requires pre-computed normal vectors for the "
                         "target point cloud")
    M0 = np.ascontiguousarray(np.eye(4) if init is None else np.asarray(init, dtype=np.float64).reshape(4, 4))
    out = np.zeros(16)
    fit, rmse, it = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    with eng._lock:
        _lib.check(eng._L.sl_icp_point_to_plane(eng._ctx, _ptr(S) if len(S) else None, S.shape[0],
                                                _ptr(T) if len(T) else None, _ptr(N) if len(N) else None,
                                                T.shape[0], float(max_correspondence_distance), M0.ctypes.data,
                                                int(max_iteration), float(relative_fitness), float(relative_rmse),
                                                out.ctypes.data, ctypes.byref(fit), ctypes.byref(rmse),
                                                ctypes.byref(it), eng._stream(None)),
                   eng._ctx, "sl_icp_point_to_plane")
    return {"transformation": out.reshape(4, 4), "fitness": fit.value, "inlier_rmse": rmse.value,
            "iterations": it.value}


def radius_search(points, radius: float, max_nn: int, *, device=None):
    """KDTreeFlann.search_hybrid_vector_3d of every point (sl_radius_search)
    -> (idx int32 [N, max_nn], d2 f64 [N, max_nn], count int32 [N]) on the
    device; row i's first count[i] entries, ascending (d2, index)."""
    eng = _engine(device)
    P = _f64(points, eng.device)
    n = P.shape[0]
    idx = torch.empty((max(n, 1), max_nn), dtype=torch.int32, device=eng.device)
    d2 = torch.empty((max(n, 1), max_nn), dtype=torch.float64, device=eng.device)
    cnt = torch.empty(max(n, 1), dtype=torch.int32, device=eng.device)
    with eng._lock:
        _lib.check(eng._L.sl_radius_search(eng._ctx, _ptr(P), n, float(radius), int(max_nn), idx.data_ptr(),
                                           d2.data_ptr(), cnt.data_ptr(), eng._stream(None)),
                   eng._ctx, "sl_radius_search")
    return idx[:n], d2[:n], cnt[:n]


def compute_fpfh_feature(points, normals, radius: float, max_nn: int = 100, *, device=None) -> torch.Tensor:
    """o3d.pipelines.registration.compute_fpfh_feature(pcd,
    KDTreeSearchParamHybrid(radius, max_nn)) (processing.py:91-94) ->
    features f64 [N, 33] on the device (Open3D's Feature.data transposed)."""
    eng = _engine(device)
    P = _f64(points, eng.device)
    N = _f64(normals, eng.device)
    if N.shape != P.shape:
        raise ValueError("compute_fpfh_feature needs a normal per point")
    n = P.shape[0]
    out = torch.empty((max(n, 1), 33), dtype=torch.float64, device=eng.device)
    with eng._lock:
        _lib.check(eng._L.sl_compute_fpfh(eng._ctx, _ptr(P), _ptr(N), n, float(radius), int(max_nn), out.data_ptr(),
                                          eng._stream(None)), eng._ctx, "sl_compute_fpfh")
    return out[:n]


def feature_nn(a, b, *, device=None) -> torch.Tensor:
    """Nearest row of ``b`` for every row of ``a`` (33-D features,
    sl_feature_nn) -> int32 [len(a)] on the device."""
    eng = _engine(device)
    A = torch.as_tensor(a).to(device=eng.device, dtype=torch.float64).contiguous()
    B = torch.as_tensor(b).to(device=eng.device, dtype=torch.float64).contiguous()
    if A.dim() != 2 or B.dim() != 2 or A.shape[1] != 33 or B.shape[1] != 33:
        raise ValueError("features must be [N, 33]")
    out = torch.empty(max(A.shape[0], 1), dtype=torch.int32, device=eng.device)
    with eng._lock:
        _lib.check(eng._L.sl_feature_nn(eng._ctx, _ptr(A), A.shape[0], _ptr(B), B.shape[0], 33, out.data_ptr(),
                                        eng._stream(None)), eng._ctx, "sl_feature_nn")
    return out[:A.shape[0]]


def registration_ransac_based_on_feature_matching(source, target, source_feature, target_feature,
                                                  mutual_filter: bool, max_correspondence_distance: float, *,
                                                  edge_similarity: float = 0.9, max_iteration: int = 100000,
                                                  confidence: float = 0.999, seed: int = 0, device=None) -> dict:
    """o3d.pipelines.registration.registration_ransac_based_on_feature_matching
    (source, target, source_fpfh, target_fpfh, mutual_filter,
    max_correspondence_distance, TransformationEstimationPointToPoint(False),
    3, [CorrespondenceCheckerBasedOnEdgeLength(edge_similarity),
    CorrespondenceCheckerBasedOnDistance(max_correspondence_distance)],
    RANSACConvergenceCriteria(max_iteration, confidence)) (processing.py:
    98-111) on the GPU (sl_ransac_feature_matching; ``seed`` fixes the draw,
    which Open3D leaves unseeded) -> {"transformation": 4x4 numpy, "fitness",
    "inlier_rmse", "iterations", "validations", "correspondences"}."""
    eng = _engine(device)
    S = _f64(source, eng.device)
    T = _f64(target, eng.device)
    FS = torch.as_tensor(source_feature).to(device=eng.device, dtype=torch.float64).contiguous()
    FT = torch.as_tensor(target_feature).to(device=eng.device, dtype=torch.float64).contiguous()
    if FS.shape != (S.shape[0], 33) or FT.shape != (T.shape[0], 33):
        raise ValueError("features must be [N, 33], one row per point")
    out = np.zeros(16)
    fit, rmse = ctypes.c_double(), ctypes.c_double()
    it, vals, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    with eng._lock:
        _lib.check(eng._L.sl_ransac_feature_matching(
            eng._ctx, _ptr(S) if len(S) else None, S.shape[0], _ptr(T) if len(T) else None, T.shape[0],
            _ptr(FS) if len(FS) else None, _ptr(FT) if len(FT) else None, int(bool(mutual_filter)),
            float(max_correspondence_distance), float(edge_similarity), int(max_iteration), float(confidence),
            int(seed) & ((1 << 64) - 1), out.ctypes.data, ctypes.byref(fit), ctypes.byref(rmse), ctypes.byref(it),
            ctypes.byref(vals), ctypes.byref(nc), eng._stream(None)), eng._ctx, "sl_ransac_feature_matching")
    return {"transformation": out.reshape(4, 4), "fitness": fit.value, "inlier_rmse": rmse.value,
            "iterations": it.value, "validations": vals.value, "correspondences": nc.value}


def preprocess_point_cloud(points, voxel_size: float, *, device=None):
    """preprocess_point_cloud (processing.py:79-96): voxel_down_sample, normals
    (radius 2 voxel, max_nn 30), FPFH (radius 5 voxel, max_nn 100) ->
    (down points, their normals, their features) on the device."""
    Pd, _ = voxel_down_sample(points, None, voxel_size, device=device)
    Nd = estimate_normals(Pd, voxel_size * 2, 30, device=device)
    Fd = compute_fpfh_feature(Pd, Nd, voxel_size * 5, 100, device=device)
    return Pd, Nd, Fd


def execute_global_registration(source_down, target_down, source_fpfh, target_fpfh, voxel_size: float, *,
                                seed: int = 0, device=None) -> dict:
    """execute_global_registration (processing.py:98-113): RANSAC on FPFH
    matches with the reference's settings (mutual filter, distance 1.5 voxel,
    edge length 0.9, 100000 iterations, confidence 0.999)."""
    return registration_ransac_based_on_feature_matching(
        source_down, target_down, source_fpfh, target_fpfh, True, voxel_size * 1.5, edge_similarity=0.9,
        max_iteration=100000, confidence=0.999, seed=seed, device=device)


def rigid_inverse(M) -> np.ndarray:
    """[R | t]^-1 = [R^T | -(R^T t)] of a rigid 4x4 pose."""
    M = np.asarray(M, dtype=np.float64).reshape(4, 4)
    R, t = M[:3, :3], M[:3, 3]
    out = np.zeros((4, 4))
    out[:3, :3] = R.T
    for i in range(3):
        out[i, 3] = -((R[0, i] * t[0] + R[1, i] * t[1]) + R[2, i] * t[2])
    out[3, 3] = 1.0
    return out


def mat4(a, b) -> np.ndarray:
    """Row-major 4x4 product ((a0 b0 + a1 b1) + a2 b2) + a3 b3 (np.dot of
    processing.py:162, in a fixed order)."""
    a = np.asarray(a, dtype=np.float64).reshape(4, 4)
    b = np.asarray(b, dtype=np.float64).reshape(4, 4)
    out = np.empty((4, 4))
    for i in range(4):
        for j in range(4):
            out[i, j] = ((a[i, 0] * b[0, j] + a[i, 1] * b[1, j]) + a[i, 2] * b[2, j]) + a[i, 3] * b[3, j]
    return out


def merge_pro_360(input_folder, output_path, voxel_size: float = 0.02, *, seed_poses=None, device=None,
                  binary: bool = True, order: str = "lexicographic", max_iteration: int = 30,
                  return_transforms: bool = False, ransac_seed: int = 0):
    """merge_pro_360 (processing.py:116-182): the clouds of ``input_folder``
    (``ply_files(order)``; default the reference's lexicographic order)
    registered in sequence -- scan i onto scan i-1 by point-to-plane ICP
    between their voxel-downsampled clouds (target normals radius 2 voxel,
    max_nn 30; max correspondence distance = voxel_size; :145-157), the
    transforms accumulated T_i = T_{i-1} T_local (:159-167) and scan i moved
    by T_i -- then merged, voxel-downsampled, outlier-filtered, normals
    estimated and written in Open3D's layout (as merge_pro_360_posed).

    Each ICP starts, as the reference's, from the FPFH + RANSAC global
    estimate (preprocess_point_cloud / execute_global_registration, :79-113:
    FPFH radius 5 voxel, RANSAC distance 1.5 voxel; ``ransac_seed`` fixes its
    draw), unless ``seed_poses`` is given: then from ``inverse(seed_poses[i-1])
    @ seed_poses[i]`` (the turntable's relative pose between the two views;
    poses mapping each view into a common frame, e.g. synth.turntable_pose).
    Returns (points, colors, normals) on the device (+ the accumulated
    transforms with ``return_transforms``)."""
    print(f"[Merge 360] Loading clouds from {input_folder}...")
    files = ply_files(input_folder, order)
    if len(files) < 2:
        raise ValueError("Need at least 2 .ply files to merge.")
    if seed_poses is not None:
        seed_poses = np.asarray(seed_poses, dtype=np.float64).reshape(-1, 4, 4)
        if len(seed_poses) != len(files):
            raise ValueError(f"{len(files)} clouds but {len(seed_poses)} seed poses")
    eng = _engine(device)
    pcds = []
    for f in files:
        P, C = ply.read_ply(f)
        pcds.append((torch.from_numpy(np.ascontiguousarray(P, dtype=np.float64)).to(eng.device),
                     torch.from_numpy(np.ascontiguousarray(C)).to(eng.device)))
    print(f"[Merge 360] Loaded {len(pcds)} clouds. Running Sequential Registration (New360 Logic)...")
    down = {}

    def prep(i):  # preprocess_point_cloud (:79-96); the FPFH features only for RANSAC
        if i not in down:
            if seed_poses is None:
                down[i] = preprocess_point_cloud(pcds[i][0], voxel_size, device=eng.device)
            else:
                Pd, _ = voxel_down_sample(pcds[i][0], None, voxel_size, device=eng.device)
                down[i] = (Pd, estimate_normals(Pd, voxel_size * 2, 30, device=eng.device), None)
        return down[i]
    accum = np.eye(4)
    transforms = [accum.copy()]
    parts_p, parts_c = [pcds[0][0]], [pcds[0][1]]
    for i in range(1, len(pcds)):
        print(f"[Merge 360] Aligning Scan {i} -> Scan {i-1}...")
        src, _, src_f = prep(i)
        tgt, tgt_n, tgt_f = prep(i - 1)
        if seed_poses is None:  # execute_global_registration (:146-151)
            init = execute_global_registration(src, tgt, src_f, tgt_f, voxel_size, seed=ransac_seed + i,
                                               device=eng.device)["transformation"]
        else:
            init = mat4(rigid_inverse(seed_poses[i - 1]), seed_poses[i])
        T_local = registration_icp(src, tgt, tgt_n, voxel_size, init, max_iteration=max_iteration,
                                   device=eng.device)["transformation"]
        accum = mat4(accum, T_local)
        transforms.append(accum.copy())
        parts_p.append(transform(pcds[i][0], accum, device=eng.device))
        parts_c.append(pcds[i][1])
        down.pop(i - 1, None)
    merged_p = torch.cat(parts_p)
    merged_c = torch.cat(parts_c)
    print("[Merge 360] Post-processing (Downsample + Outlier removal)...")
    P, C = postprocess(merged_p, merged_c, voxel_size, device=eng.device)
    N = estimate_normals(P, voxel_size * 2, 30, device=eng.device)
    ply.save_ply_open3d(P.cpu().numpy(), C.cpu().numpy(), output_path, normals=N.cpu().numpy(), binary=binary)
    print(f"[Merge 360] Saved merged cloud to {output_path}")
    return (P, C, N, transforms) if return_transforms else (P, C, N)


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
