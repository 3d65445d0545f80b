"""CPU restatement of the merge stage's point-cloud filters -- TEST INFRASTRUCTURE.

Only tests/ import this.  It restates, in NumPy, the two Open3D calls that
server/processing.py:171-175 (merge_pro_360) and :64 (remove_outliers) make:

- ``PointCloud::VoxelDownSample(voxel_size)``;
- ``PointCloud::RemoveStatisticalOutliers(nb_neighbors, std_ratio)``.

Both follow Open3D's published source (open3d/geometry/PointCloud.cpp).
requirements.txt:6 lists ``open3d`` with no version pin; the two functions have
had this form since 0.10.

PARITY UNPINNED: Open3D is not installed in this image, so no Open3D output
is available to pin this restatement.  The GPU path (csrc/slmerge.hip) is
checked against it bit for bit.

Summation orders are Open3D's:
- voxel sums run in ascending point index (``AccumulatedPoint::AddPoint``);
- a point's kNN distances are ``std::accumulate``'d in ascending order;
- the cloud mean / variance are sequential (``std::accumulate`` /
  ``std::inner_product``).

Squared distances use nanoflann's ``L2_Adaptor`` order for three dimensions:
``((dx*dx) + dy*dy) + dz*dz`` with ``d = query - point``.  Colours are Open3D's
doubles c/255 and are written back as ``round(clamp(c) * 255)``.

Voxel output order is ascending voxel key (ix, iy, iz); Open3D's is its hash
map's iteration order.
"""
from __future__ import annotations

import numpy as np


def _round_half_away(x):
    """std::round for x >= 0, exactly (trunc + fraction test, no x + 0.5 rounding)."""
    r = np.trunc(x)
    return r + ((x - r) >= 0.5)


def voxel_down_sample(points, colors, voxel_size):
    """-> (points f64 (M,3), colors uint8 (M,3) or None) in ascending voxel key."""
    P = np.asarray(points, dtype=np.float64)
    if voxel_size <= 0.0:
        raise ValueError("voxel_size <= 0.")
    if len(P) == 0:
        return np.zeros((0, 3)), (None if colors is None else np.zeros((0, 3), np.uint8))
    mn, mx = P.min(0), P.max(0)
    lo = mn - voxel_size * 0.5
    hi = mx + voxel_size * 0.5
    if voxel_size * float(2 ** 31 - 1) < (hi - lo).max():
        raise ValueError("voxel_size is too small.")
    idx = np.floor((P - lo) / voxel_size).astype(np.int64)
    dims = np.floor((mx - lo) / voxel_size).astype(np.int64) + 1
    key = (idx[:, 0] * dims[1] + idx[:, 1]) * dims[2] + idx[:, 2]
    uk, inv = np.unique(key, return_inverse=True)
    m = len(uk)
    S = np.zeros((m, 3))
    np.add.at(S, inv, P)  # unbuffered, in index order: Open3D's AddPoint sequence
    cnt = np.bincount(inv, minlength=m).astype(np.float64)
    out = S / cnt[:, None]
    oc = None
    if colors is not None:
        Cs = np.zeros((m, 3))
        np.add.at(Cs, inv, np.asarray(colors, dtype=np.float64) / 255.0)
        avg = Cs / cnt[:, None]
        oc = _round_half_away(np.clip(avg, 0.0, 1.0) * 255.0).astype(np.uint8)
    return out, oc


def knn_mean_distances(points, nb_neighbors, chunk=512):
    """Mean of the square roots of the nb_neighbors smallest squared distances
    (the point itself included), accumulated in ascending order.  Brute force:
    small clouds only."""
    P = np.asarray(points, dtype=np.float64)
    n = len(P)
    kk = min(nb_neighbors, n)
    avg = np.empty(n)
    for a in range(0, n, chunk):
        q = P[a:a + chunk]
        d0 = q[:, None, 0] - P[None, :, 0]
        d1 = q[:, None, 1] - P[None, :, 1]
        d2 = q[:, None, 2] - P[None, :, 2]
        dd = (d0 * d0 + d1 * d1) + d2 * d2
        part = np.sort(np.partition(dd, kk - 1, axis=1)[:, :kk], axis=1)
        avg[a:a + chunk] = np.cumsum(np.sqrt(part), axis=1)[:, -1] / kk
    return avg


def statistical_outlier_indices(avg, std_ratio):
    """RemoveStatisticalOutliers' selection from the per-point means."""
    avg = np.asarray(avg, dtype=np.float64)
    n = len(avg)
    if n == 0:
        return np.zeros(0, np.int64)
    pos = avg[avg > 0]
    mean = (np.cumsum(pos)[-1] if len(pos) else 0.0) / n
    terms = np.where(avg > 0, (avg - mean) * (avg - mean), 0.0)
    sq = np.cumsum(terms)[-1]
    with np.errstate(divide="ignore", invalid="ignore"):
        std = np.sqrt(sq / (n - 1)) if n > 1 else np.float64(np.nan)
    thr = mean + std_ratio * std
    return np.flatnonzero((avg > 0) & (avg < thr)).astype(np.int64)


def remove_statistical_outlier(points, nb_neighbors, std_ratio):
    """-> (indices kept, per-point mean kNN distance)."""
    avg = knn_mean_distances(points, nb_neighbors)
    return statistical_outlier_indices(avg, std_ratio), avg
