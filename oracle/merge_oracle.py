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


# --------------------------------------------------------------------------
# PointCloud::EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn)), the
# call server/processing.py:178 makes on the merged cloud (radius = 2 voxel,
# max_nn = 30), restated from Open3D's published source
# (geometry/EstimateNormals.cpp, utility/Eigen.cpp ComputeCovariance,
# KDTreeFlann::SearchHybrid):
#
# - neighbours: every point with ((dx*dx + dy*dy) + dz*dz) < radius^2 (the
#   point itself included), ascending distance, the first max_nn (ties by
#   ascending index here; nanoflann's std::sort leaves them unordered);
# - fewer than 3 neighbours -> covariance = identity, else the cumulants
#   (sum x, y, z, xx, xy, xz, yy, yz, zz in neighbour order) / count and
#   covariance = E[ab] - E[a] E[b];
# - normal = FastEigen3x3(covariance) (Geometric Tools' robust symmetric 3x3
#   eigen solver: eigenvector of the smallest eigenvalue); zero -> (0, 0, 1).
#
# FastEigen3x3 calls std::acos / std::cos.  Their last-ulp behaviour is the
# C library's, so the GPU path and this restatement both use the fdlibm
# algorithms below (only +, -, *, /, sqrt and bit masking: bit-identical on
# any IEEE machine); they differ from glibc's by at most an ulp or so.  Parity
# with Open3D stays unpinned (no Open3D in this image).
# --------------------------------------------------------------------------
import math  # noqa: E402
import struct  # noqa: E402

_PIO2_HI = 1.57079632679489655800e+00
_PIO2_LO = 6.12323399573676603587e-17
_PI = 3.14159265358979311600e+00
_PS = (1.66666666666666657415e-01, -3.25565818622400915405e-01, 2.01212532134862925881e-01,
       -4.00555345006794114027e-02, 7.91534994289814532176e-04, 3.47933107596021167570e-05)
_QS = (-2.40339491173441421878e+00, 2.02094576023350569471e+00, -6.88283971605453293030e-01,
       7.70381505559019352791e-02)
_C = (4.16666666666666019037e-02, -1.38888888888741095749e-03, 2.48015872894767294178e-05,
      -2.75573143513906633035e-07, 2.08757232129817482790e-09, -1.13596475577881948265e-11)
_S = (-1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04,
      2.75573137070700676789e-06, -2.50507602534068634195e-08, 1.58969099521155010221e-10)
_INVPIO2 = 6.36619772367581382433e-01
_PIO2_1 = 1.57079632673412561417e+00
_PIO2_1T = 6.07710050650619224932e-11


def _low_word_zero(x):
    (u,) = struct.unpack("<Q", struct.pack("<d", x))
    return struct.unpack("<d", struct.pack("<Q", u & 0xFFFFFFFF00000000))[0]


def _acos_rational(z):
    p = z * (_PS[0] + z * (_PS[1] + z * (_PS[2] + z * (_PS[3] + z * (_PS[4] + z * _PS[5])))))
    q = 1.0 + z * (_QS[0] + z * (_QS[1] + z * (_QS[2] + z * _QS[3])))
    return p / q


def acos_det(x):
    """fdlibm e_acos.c for x in [-1, 1]."""
    ax = abs(x)
    if ax >= 1.0:
        return 0.0 if x == 1.0 else (_PI if x == -1.0 else float("nan"))
    if ax < 0.5:
        if ax <= 2.0 ** -57:
            return _PIO2_HI + _PIO2_LO
        r = _acos_rational(x * x)
        return _PIO2_HI - (x - (_PIO2_LO - x * r))
    if x < 0.0:
        z = (1.0 + x) * 0.5
        s = math.sqrt(z)
        r = _acos_rational(z)
        w = r * s - _PIO2_LO
        return _PI - 2.0 * (s + w)
    z = (1.0 - x) * 0.5
    s = math.sqrt(z)
    df = _low_word_zero(s)
    c = (z - df * df) / (s + df)
    r = _acos_rational(z)
    w = r * s + c
    return 2.0 * (df + w)


def _kcos(x, y):
    z = x * x
    w = z * z
    r = z * (_C[0] + z * (_C[1] + z * _C[2])) + w * w * (_C[3] + z * (_C[4] + z * _C[5]))
    hz = 0.5 * z
    w = 1.0 - hz
    return w + (((1.0 - w) - hz) + (z * r - x * y))


def _ksin(x, y):
    z = x * x
    w = z * z
    r = _S[1] + z * (_S[2] + z * _S[3]) + z * w * (_S[4] + z * _S[5])
    v = z * x
    return x - ((z * (0.5 * y - v * r) - y) - v * _S[0])


def cos_det(x):
    """fdlibm s_cos.c for x in [0, 4]: one-constant Cody-Waite reduction by
    pi/2 (n * _PIO2_1 is exact for n < 2^20), then the kernels."""
    if x <= 0.7853981633974483:
        return _kcos(x, 0.0)
    n = math.floor(x * _INVPIO2 + 0.5)
    fn = float(n)
    r = x - fn * _PIO2_1
    w = fn * _PIO2_1T
    y0 = r - w
    y1 = (r - y0) - w
    q = n & 3
    if q == 0:
        return _kcos(y0, y1)
    if q == 1:
        return -_ksin(y0, y1)
    if q == 2:
        return -_kcos(y0, y1)
    return _ksin(y0, y1)


def _cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def _dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def _evec0(A, e):
    r0 = (A[0][0] - e, A[0][1], A[0][2])
    r1 = (A[0][1], A[1][1] - e, A[1][2])
    r2 = (A[0][2], A[1][2], A[2][2] - e)
    c01, c02, c12 = _cross(r0, r1), _cross(r0, r2), _cross(r1, r2)
    d0, d1, d2 = _dot(c01, c01), _dot(c02, c02), _dot(c12, c12)
    dmax, imax = d0, 0
    if d1 > dmax:
        dmax, imax = d1, 1
    if d2 > dmax:
        imax = 2
    v, d = ((c01, d0), (c02, d1), (c12, d2))[imax]
    s = math.sqrt(d)
    return (v[0] / s, v[1] / s, v[2] / s)


def _evec1(A, ev0, e1):
    if abs(ev0[0]) > abs(ev0[1]):
        inv = 1.0 / math.sqrt(ev0[0] * ev0[0] + ev0[2] * ev0[2])
        U = (-ev0[2] * inv, 0.0, ev0[0] * inv)
    else:
        inv = 1.0 / math.sqrt(ev0[1] * ev0[1] + ev0[2] * ev0[2])
        U = (0.0, ev0[2] * inv, -ev0[1] * inv)
    V = _cross(ev0, U)
    AU = (A[0][0] * U[0] + A[0][1] * U[1] + A[0][2] * U[2],
          A[0][1] * U[0] + A[1][1] * U[1] + A[1][2] * U[2],
          A[0][2] * U[0] + A[1][2] * U[1] + A[2][2] * U[2])
    AV = (A[0][0] * V[0] + A[0][1] * V[1] + A[0][2] * V[2],
          A[0][1] * V[0] + A[1][1] * V[1] + A[1][2] * V[2],
          A[0][2] * V[0] + A[1][2] * V[1] + A[2][2] * V[2])
    m00 = U[0] * AU[0] + U[1] * AU[1] + U[2] * AU[2] - e1
    m01 = U[0] * AV[0] + U[1] * AV[1] + U[2] * AV[2]
    m11 = V[0] * AV[0] + V[1] * AV[1] + V[2] * AV[2] - e1
    a00, a01, a11 = abs(m00), abs(m01), abs(m11)
    if a00 >= a11:
        if max(a00, a01) > 0.0:
            if a00 >= a01:
                m01 /= m00
                m00 = 1.0 / math.sqrt(1.0 + m01 * m01)
                m01 *= m00
            else:
                m00 /= m01
                m01 = 1.0 / math.sqrt(1.0 + m00 * m00)
                m00 *= m01
            return (m01 * U[0] - m00 * V[0], m01 * U[1] - m00 * V[1], m01 * U[2] - m00 * V[2])
        return U
    if max(a11, a01) > 0.0:
        if a11 >= a01:
            m01 /= m11
            m11 = 1.0 / math.sqrt(1.0 + m01 * m01)
            m01 *= m11
        else:
            m11 /= m01
            m01 = 1.0 / math.sqrt(1.0 + m11 * m11)
            m11 *= m01
        return (m11 * U[0] - m01 * V[0], m11 * U[1] - m01 * V[1], m11 * U[2] - m01 * V[2])
    return U


def fast_eigen3x3(C):
    """Open3D's FastEigen3x3: unit eigenvector of the smallest eigenvalue of
    the symmetric 3x3 C (tuple of rows); (0, 0, 0) for C == 0."""
    mx = max(C[0][0], C[0][1], C[0][2], C[1][0], C[1][1], C[1][2], C[2][0], C[2][1], C[2][2])
    if mx == 0.0:
        return (0.0, 0.0, 0.0)
    A = [[C[r][k] / mx for k in range(3)] for r in range(3)]
    norm = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2]
    if norm > 0.0:
        q = (A[0][0] + A[1][1] + A[2][2]) / 3.0
        b00, b11, b22 = A[0][0] - q, A[1][1] - q, A[2][2] - q
        p = math.sqrt((b00 * b00 + b11 * b11 + b22 * b22 + norm * 2.0) / 6.0)
        c00 = b11 * b22 - A[1][2] * A[1][2]
        c01 = A[0][1] * b22 - A[1][2] * A[0][2]
        c02 = A[0][1] * A[1][2] - b11 * A[0][2]
        det = (b00 * c00 - A[0][1] * c01 + A[0][2] * c02) / (p * p * p)
        half_det = min(max(det * 0.5, -1.0), 1.0)
        angle = acos_det(half_det) / 3.0
        two_thirds_pi = 2.09439510239319549
        beta2 = cos_det(angle) * 2.0
        beta0 = cos_det(angle + two_thirds_pi) * 2.0
        beta1 = -(beta0 + beta2)
        ev = (q + p * beta0, q + p * beta1, q + p * beta2)
        if half_det >= 0.0:
            e2 = _evec0(A, ev[2])
            if ev[2] < ev[0] and ev[2] < ev[1]:
                return e2
            e1 = _evec1(A, e2, ev[1])
            if ev[1] < ev[0] and ev[1] < ev[2]:
                return e1
            return _cross(e1, e2)
        e0 = _evec0(A, ev[0])
        if ev[0] < ev[1] and ev[0] < ev[2]:
            return e0
        e1 = _evec1(A, e0, ev[1])
        if ev[1] < ev[0] and ev[1] < ev[2]:
            return e1
        return _cross(e0, e1)
    if C[0][0] < C[1][1] and C[0][0] < C[2][2]:
        return (1.0, 0.0, 0.0)
    if C[1][1] < C[0][0] and C[1][1] < C[2][2]:
        return (0.0, 1.0, 0.0)
    return (0.0, 0.0, 1.0)


def hybrid_neighbours(points, radius, max_nn):
    """KDTreeFlann::SearchHybrid for every point -> list of index arrays
    (ascending (distance, index)), exact distances in nanoflann's order
    (which compares against radius * radius: a negative radius acts as its
    absolute value)."""
    from scipy.spatial import cKDTree
    P = np.asarray(points, dtype=np.float64)
    r2 = radius * radius
    cand = cKDTree(P).query_ball_point(P, abs(radius) * (1.0 + 1e-9) + 1e-300)
    out = []
    for i, c in enumerate(cand):
        c = np.asarray(sorted(c), dtype=np.int64)
        d = P[i] - P[c]
        d2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        keep = d2 < r2
        c, d2 = c[keep], d2[keep]
        o = np.lexsort((c, d2))
        out.append(c[o][:max_nn])
    return out


def estimate_normals(points, radius, max_nn=30):
    """PointCloud::EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn))
    on a cloud without normals -> (N, 3) float64."""
    P = np.asarray(points, dtype=np.float64)
    out = np.empty_like(P)
    for i, nb in enumerate(hybrid_neighbours(P, radius, max_nn)):
        if len(nb) >= 3:
            s = [0.0] * 9
            for j in nb.tolist():
                x, y, z = P[j].tolist()
                s[0] += x
                s[1] += y
                s[2] += z
                s[3] += x * x
                s[4] += x * y
                s[5] += x * z
                s[6] += y * y
                s[7] += y * z
                s[8] += z * z
            k = float(len(nb))
            s = [v / k for v in s]
            c01 = s[4] - s[0] * s[1]
            c02 = s[5] - s[0] * s[2]
            c12 = s[7] - s[1] * s[2]
            C = ((s[3] - s[0] * s[0], c01, c02), (c01, s[6] - s[1] * s[1], c12), (c02, c12, s[8] - s[2] * s[2]))
        else:
            C = ((1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))
        n = fast_eigen3x3(C)
        if math.sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]) == 0.0:
            n = (0.0, 0.0, 1.0)
        out[i] = n
    return out


# ---------------------------------------------------------------- ICP ----
# registration_icp(source_down, target_down, voxel_size, init,
# TransformationEstimationPointToPlane()) of merge_pro_360
# (server/processing.py:154-156) -- Open3D's RegistrationICP loop
# (open3d/pipelines/registration/Registration.cpp) and the point-to-plane
# step (TransformationEstimation.cpp, utility/Eigen.cpp), restated with the
# arithmetic order csrc/slmerge.hip's sl_icp_point_to_plane fixes:
#   - correspondence of a moved source point q: the target point of least
#     (d2, index) with d2 = ((dx*dx) + dy*dy) + dz*dz < max_distance**2
#     (nanoflann's strict radius test; Open3D breaks distance ties arbitrarily);
#   - r = ((e0 n0 + e1 n1) + e2 n2), e = q - t, J = (q x n, n); JTJ (upper
#     triangle, row-major), JTr, sum d2, count folded left to right over
#     64-source-point blocks, then the blocks left to right (Open3D: an
#     OpenMP reduction, order unspecified);
#   - 6x6 pivoted LDLT as Eigen's (Open3D: A.ldlt().solve(b)), zero pivots
#     -> zero components; x = (alpha, beta, gamma, tx, ty, tz) -> [Rz Ry Rx | t]
#     (TransformVector6dToMatrix4d), products ((a0 b0 + a1 b1) + a2 b2)
#     [+ a3 b3];
#   - transformation = update @ transformation; the source is moved by the
#     update each step (PointCloud::Transform, row order ((m0 x + m1 y) +
#     m2 z) + m3); init applied first unless exactly the identity;
#   - stop when |d fitness| < relative_fitness and |d rmse| < relative_rmse.
# PARITY UNPINNED (no Open3D in this image): the GPU matches this restatement.
ICP_BLOCK = 64


def _transform(P, M):
    x, y, z = P[:, 0], P[:, 1], P[:, 2]
    out = np.empty_like(P)
    for r in range(3):
        out[:, r] = ((M[r][0] * x + M[r][1] * y) + M[r][2] * z) + M[r][3]
    return out


def icp_correspondences(Q, target, max_distance):
    """-> (corr int64 [n] (-1: none), d2 f64 [n])."""
    from scipy.spatial import cKDTree
    T = np.asarray(target, dtype=np.float64)
    r2 = max_distance * max_distance
    tree = cKDTree(T)
    corr = np.full(len(Q), -1, dtype=np.int64)
    d2 = np.zeros(len(Q))
    cand = tree.query_ball_point(Q, max_distance * (1.0 + 1e-9) + 1e-300)
    for i, c in enumerate(cand):
        if not c:
            continue
        c = np.asarray(sorted(c), dtype=np.int64)
        d = Q[i] - T[c]
        dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        ok = dd < r2
        if not ok.any():
            continue
        c, dd = c[ok], dd[ok]
        k = np.lexsort((c, dd))[0]
        corr[i] = c[k]
        d2[i] = dd[k]
    return corr, d2


def icp_sums(Q, target, normals, corr, d2):
    """The 29 folded sums (JTJ upper 21, JTr 6, sum d2, count)."""
    T = np.asarray(target, dtype=np.float64)
    N = np.asarray(normals, dtype=np.float64)
    n = len(Q)
    ok = corr >= 0
    j = np.where(ok, corr, 0)
    s0, s1, s2 = Q[:, 0], Q[:, 1], Q[:, 2]
    n0, n1, n2 = N[j, 0], N[j, 1], N[j, 2]
    e0, e1, e2 = s0 - T[j, 0], s1 - T[j, 1], s2 - T[j, 2]
    r = (e0 * n0 + e1 * n1) + e2 * n2
    J = [s1 * n2 - s2 * n1, s2 * n0 - s0 * n2, s0 * n1 - s1 * n0, n0, n1, n2]
    cols = []
    for a in range(6):
        for c in range(a, 6):
            cols.append(J[a] * J[c])
    for a in range(6):
        cols.append(J[a] * r)
    cols.append(d2)
    cols.append(np.ones(n))
    C = np.stack(cols, axis=1)
    C[~ok] = 0.0  # skipped points: adding +0.0 to an accumulator that starts at +0.0
    nb = (n + ICP_BLOCK - 1) // ICP_BLOCK
    pad = np.zeros((nb * ICP_BLOCK, C.shape[1]))
    pad[:n] = C
    part = np.cumsum(pad.reshape(nb, ICP_BLOCK, -1), axis=1)[:, -1, :]  # left fold inside each block
    out = [0.0] * C.shape[1]
    for b in range(nb):  # blocks left to right
        for k in range(C.shape[1]):
            out[k] = out[k] + float(part[b, k])
    return out


def _mat3(a, b):
    return [[(a[i][0] * b[0][j] + a[i][1] * b[1][j]) + a[i][2] * b[2][j] for j in range(3)] for i in range(3)]


def mat4(a, b):
    """Row-major 4x4 product, ((a0 b0 + a1 b1) + a2 b2) + a3 b3."""
    return [[((a[i][0] * b[0][j] + a[i][1] * b[1][j]) + a[i][2] * b[2][j]) + a[i][3] * b[3][j]
             for j in range(4)] for i in range(4)]


def icp_update(sums):
    """JTJ x = -JTr -> the 4x4 update, as Open3D's SolveLinearSystemPSD
    (x = A.ldlt().solve(b), no PSD checks): Eigen's LDLT -- left-looking,
    diagonal pivoting on the largest |a_ii| not yet factored (first on ties),
    zero pivots left unscaled, and D's pseudo-inverse in the solve (components
    with |d_i| <= DBL_MIN are 0).  Sums of products left to right (Eigen's
    vectorised order may differ in the last bits).  Identity only when the
    solution is not finite."""
    import math
    import sys
    M = [[0.0] * 6 for _ in range(6)]
    k = 0
    for a in range(6):
        for c in range(a, 6):
            M[a][c] = M[c][a] = sums[k]
            k += 1
    b = [-sums[21 + a] for a in range(6)]
    ident = [[1.0 if i == j else 0.0 for j in range(4)] for i in range(4)]
    tr = [0] * 6
    zero_all = False
    for j in range(6):
        p = j
        for i in range(j + 1, 6):
            if abs(M[i][i]) > abs(M[p][p]):
                p = i
        tr[j] = p
        if p != j:
            M[j], M[p] = M[p], M[j]
            for row in M:
                row[j], row[p] = row[p], row[j]
        if j > 0:
            tmp = [M[q][q] * M[j][q] for q in range(j)]
            d = 0.0
            for q in range(j):
                d = d + M[j][q] * tmp[q]
            M[j][j] = M[j][j] - d
            for i in range(j + 1, 6):
                v = 0.0
                for q in range(j):
                    v = v + M[i][q] * tmp[q]
                M[i][j] = M[i][j] - v
        piv = M[j][j]
        if j == 0 and not (abs(piv) > 0.0):
            zero_all = True
            break
        if abs(piv) > 0.0:
            for i in range(j + 1, 6):
                M[i][j] = M[i][j] / piv
    if zero_all:
        x = [0.0] * 6
    else:
        for j in range(6):
            b[j], b[tr[j]] = b[tr[j]], b[j]
        for i in range(6):
            v = 0.0
            for q in range(i):
                v = v + M[i][q] * b[q]
            b[i] = b[i] - v
        for i in range(6):
            b[i] = b[i] / M[i][i] if abs(M[i][i]) > sys.float_info.min else 0.0
        for i in range(5, -1, -1):
            v = 0.0
            for q in range(i + 1, 6):
                v = v + M[q][i] * b[q]
            b[i] = b[i] - v
        for j in range(5, -1, -1):
            b[j], b[tr[j]] = b[tr[j]], b[j]
        x = b
    if not all(math.isfinite(v) for v in x):
        return ident
    ca, sa, cb, sb = math.cos(x[0]), math.sin(x[0]), math.cos(x[1]), math.sin(x[1])
    cg, sg = math.cos(x[2]), math.sin(x[2])
    Rx = [[1.0, 0.0, 0.0], [0.0, ca, -sa], [0.0, sa, ca]]
    Ry = [[cb, 0.0, sb], [0.0, 1.0, 0.0], [-sb, 0.0, cb]]
    Rz = [[cg, -sg, 0.0], [sg, cg, 0.0], [0.0, 0.0, 1.0]]
    R = _mat3(Rz, _mat3(Ry, Rx))
    return [R[0] + [x[3]], R[1] + [x[4]], R[2] + [x[5]], [0.0, 0.0, 0.0, 1.0]]


def registration_icp_point_to_plane(source, target, target_normals, max_distance, init=None, max_iteration=30,
                                    relative_fitness=1e-6, relative_rmse=1e-6):
    """-> dict(transformation 4x4 (numpy), fitness, inlier_rmse, iterations)."""
    import math
    Q = np.array(source, dtype=np.float64)
    T = [[1.0 if i == j else 0.0 for j in range(4)] for i in range(4)] if init is None else \
        [[float(v) for v in row] for row in np.asarray(init, dtype=np.float64).reshape(4, 4)]
    n = len(Q)
    res = {"fitness": 0.0, "inlier_rmse": 0.0, "iterations": 0}
    if n == 0 or len(target) == 0:
        res["transformation"] = np.array(T)
        return res
    ident = all(T[i][j] == (1.0 if i == j else 0.0) for i in range(4) for j in range(4))
    if not ident:
        Q = _transform(Q, T)

    def evaluate(Q):
        corr, d2 = icp_correspondences(Q, target, max_distance)
        s = icp_sums(Q, target, target_normals, corr, d2)
        cnt = s[28]
        return s, cnt / n, (math.sqrt(s[27] / cnt) if cnt > 0.0 else 0.0)
    sums, fit, rmse = evaluate(Q)
    it_done = 0
    for it in range(max_iteration):
        U = icp_update(sums)
        T = mat4(U, T)
        Q = _transform(Q, U)
        f0, r0 = fit, rmse
        sums, fit, rmse = evaluate(Q)
        it_done = it + 1
        if abs(f0 - fit) < relative_fitness and abs(r0 - rmse) < relative_rmse:
            break
    return {"transformation": np.array(T), "fitness": fit, "inlier_rmse": rmse, "iterations": it_done}


def rigid_inverse(M):
    """[R | t]^-1 = [R^T | -(R^T t)], products ((a0 b0 + a1 b1) + a2 b2)."""
    M = np.asarray(M, dtype=np.float64).reshape(4, 4)
    R = M[:3, :3]
    t = M[:3, 3]
    out = np.zeros((4, 4))
    out[:3, :3] = R.T
    for i in range(3):
        out[i, 3] = -((R[0, i] * t[0] + R[1, i] * t[1]) + R[2, i] * t[2])
    out[3, 3] = 1.0
    return out
