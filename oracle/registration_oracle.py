"""CPU restatement of the merge stage's global registration -- TEST INFRASTRUCTURE.

Only tests/ import this.  It restates the two Open3D calls of
server/processing.py:79-113 that merge_pro_360 (:146-151) makes before its ICP:

- ``compute_fpfh_feature(pcd_down, KDTreeSearchParamHybrid(radius=5 voxel,
  max_nn=100))`` (:91-94): Open3D's pipelines/registration/Feature.cpp --
  ComputePairFeatures, ComputeSPFHFeature, ComputeFPFHFeature;
- ``registration_ransac_based_on_feature_matching(src, tgt, src_fpfh,
  tgt_fpfh, True, 1.5 voxel, TransformationEstimationPointToPoint(False), 3,
  [CorrespondenceCheckerBasedOnEdgeLength(0.9),
  CorrespondenceCheckerBasedOnDistance(1.5 voxel)],
  RANSACConvergenceCriteria(100000, 0.999))`` (:98-111): Registration.cpp
  (CorrespondencesFromFeatures with the mutual filter,
  RegistrationRANSACBasedOnCorrespondence), CorrespondenceChecker.cpp,
  TransformationEstimation.cpp (Eigen::umeyama without scaling, Eigen's
  JacobiSVD for the 3x3 cross-covariance).

requirements.txt:6 lists ``open3d`` without a version; these functions have
had this form since 0.12.  The restatement fixes what Open3D leaves to its
thread schedule or tree order, and csrc/slmerge.hip follows it exactly:

- neighbour lists are ascending (d2, index), d2 = ((dx*dx) + dy*dy) + dz*dz,
  d2 < radius**2, the first max_nn (the query itself first);
- feature-space nearest neighbours use nanoflann's L2_Adaptor order (four
  dimensions at a time: result += ((d0^2 + d1^2) + d2^2) + d3^2, then the
  33rd), ties to the lower index;
- RANSAC is Open3D's loop run on one thread (iteration order; the early exit
  at the estimated k), with a counter-based random draw (splitmix64 of the
  seed and the draw number) instead of std::mt19937 -- Open3D's draw is
  seeded from std::random_device unless o3d.utility.random.seed was called,
  so no run of it is reproducible anyway;
- sums of squared distances fold in blocks of 64 source points, left to right
  (Open3D: an OpenMP reduction in unspecified order).

PARITY UNPINNED: Open3D is not installed in this image (and RANSAC is
randomised), so no Open3D output pins this restatement.  The GPU path is
checked against it bit for bit: features, correspondences, every hypothesis's
transformation, the chosen result.
"""
from __future__ import annotations

import math
import struct

import numpy as np

from .merge_oracle import acos_det

M_PI = 3.14159265358979311600e+00

# ------------------------------------------------------------------ atan2 ----
# fdlibm s_atan.c / e_atan2.c (only IEEE +, -, *, / and bit tests: the same
# bits on the GPU, csrc/slmerge.hip's reg::atan2_det)
_ATANHI = (4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
           1.57079632679489655800e+00)
_ATANLO = (2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
           6.12323399573676603587e-17)
_AT = (3.33333333333329318027e-01, -1.99999999998764832476e-01, 1.42857142725034663711e-01,
       -1.11111104054623557880e-01, 9.09088713343650656196e-02, -7.69187620504482999495e-02,
       6.66107313738753120669e-02, -5.83357013379057348645e-02, 4.97687799461593236017e-02,
       -3.65315727442169155270e-02, 1.62858201153657823623e-02)
_PI_O_2 = 1.5707963267948965580e+00
_PI_LO = 1.2246467991473531772e-16


def _hi(x):
    (u,) = struct.unpack("<Q", struct.pack("<d", x))
    hi = u >> 32
    return hi - (1 << 32) if hi >= (1 << 31) else hi


def _lo(x):
    (u,) = struct.unpack("<Q", struct.pack("<d", x))
    return u & 0xFFFFFFFF


def atan_det(x):
    """fdlibm atan (finite x)."""
    hx = _hi(x)
    ix = hx & 0x7fffffff
    if ix >= 0x44100000:  # |x| >= 2^66
        if ix > 0x7ff00000 or (ix == 0x7ff00000 and _lo(x) != 0):
            return x + x
        return _ATANHI[3] + _ATANLO[3] if hx > 0 else -_ATANHI[3] - _ATANLO[3]
    if ix < 0x3fdc0000:  # |x| < 0.4375
        if ix < 0x3e200000:  # |x| < 2^-29
            return x
        idx = -1
    else:
        x = abs(x)
        if ix < 0x3ff30000:  # |x| < 1.1875
            if ix < 0x3fe60000:
                idx, x = 0, (2.0 * x - 1.0) / (2.0 + x)
            else:
                idx, x = 1, (x - 1.0) / (x + 1.0)
        elif ix < 0x40038000:  # |x| < 2.4375
            idx, x = 2, (x - 1.5) / (1.0 + 1.5 * x)
        else:
            idx, x = 3, -1.0 / x
    z = x * x
    w = z * z
    s1 = z * (_AT[0] + w * (_AT[2] + w * (_AT[4] + w * (_AT[6] + w * (_AT[8] + w * _AT[10])))))
    s2 = w * (_AT[1] + w * (_AT[3] + w * (_AT[5] + w * (_AT[7] + w * _AT[9]))))
    if idx < 0:
        return x - x * (s1 + s2)
    z = _ATANHI[idx] - ((x * (s1 + s2) - _ATANLO[idx]) - x)
    return -z if hx < 0 else z


def atan2_det(y, x):
    """fdlibm atan2 for finite y, x (NaN in -> NaN out)."""
    if math.isnan(x) or math.isnan(y):
        return x + y
    if x == 1.0:
        return atan_det(y)
    m = (1 if math.copysign(1.0, y) < 0 else 0) | (2 if math.copysign(1.0, x) < 0 else 0)
    if y == 0.0:
        if m in (0, 1):
            return y
        return M_PI if m == 2 else -M_PI
    if x == 0.0:
        return -_PI_O_2 if y < 0 else _PI_O_2
    k = ((_hi(y) & 0x7fffffff) - (_hi(x) & 0x7fffffff)) >> 20
    if k > 60:
        z = _PI_O_2 + 0.5 * _PI_LO
    elif x < 0 and k < -60:
        z = 0.0
    else:
        z = atan_det(abs(y / x))
    if m == 0:
        return z
    if m == 1:
        return -z
    if m == 2:
        return M_PI - (z - _PI_LO)
    return (z - _PI_LO) - M_PI


# -------------------------------------------------------------- neighbours ----
def radius_neighbours(points, radius, max_nn):
    """KDTreeFlann::SearchHybrid(p, radius, max_nn) of every point ->
    (list of index arrays, list of d2 arrays), ascending (d2, index)."""
    from scipy.spatial import cKDTree
    P = np.asarray(points, dtype=np.float64)
    r2 = radius * radius
    cand = cKDTree(P).query_ball_point(P, abs(radius) * (1.0 + 1e-9) + 1e-300)
    idx, dd = [], []
    for i, c in enumerate(cand):
        c = np.asarray(sorted(c), dtype=np.int64)
        d = P[i] - P[c]
        d2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        keep = d2 < r2
        c, d2 = c[keep], d2[keep]
        o = np.lexsort((c, d2))[:max_nn]
        idx.append(c[o])
        dd.append(d2[o])
    return idx, dd


# -------------------------------------------------------------------- FPFH ----
def _norm3(v):
    return math.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])


def _dot3(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def _cross3(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def pair_features(p1, n1, p2, n2):
    """ComputePairFeatures -> (f0 = atan2 angle, f1, f2, f3 = distance)."""
    dp = (p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2])
    f3 = _norm3(dp)
    if f3 == 0.0:
        return (0.0, 0.0, 0.0, 0.0)
    a1 = _dot3(n1, dp) / f3
    a2 = _dot3(n2, dp) / f3
    if acos_det(abs(a1)) > acos_det(abs(a2)):
        n1, n2 = n2, n1
        dp = (-dp[0], -dp[1], -dp[2])
        f2 = -a2
    else:
        f2 = a1
    v = _cross3(dp, n1)
    vn = _norm3(v)
    if vn == 0.0:
        return (0.0, 0.0, 0.0, 0.0)
    v = (v[0] / vn, v[1] / vn, v[2] / vn)
    w = _cross3(n1, v)
    f1 = _dot3(v, n2)
    f0 = atan2_det(_dot3(w, n2), _dot3(n1, n2))
    return (f0, f1, f2, f3)


def _bin11(x):
    """Open3D's floor(x) clamped to [0, 10] (NaN -> 0, as csrc's reg::bin11)."""
    if not x >= 0.0:
        return 0
    return 10 if x >= 11.0 else int(x)


def compute_fpfh(points, normals, radius, max_nn=100):
    """compute_fpfh_feature(pcd, KDTreeSearchParamHybrid(radius, max_nn)) ->
    (N, 33) float64 (Open3D's Feature.data_ transposed)."""
    P = np.asarray(points, dtype=np.float64)
    Nn = np.asarray(normals, dtype=np.float64)
    n = len(P)
    nbr, d2 = radius_neighbours(P, radius, max_nn)
    spfh = np.zeros((n, 33))
    Pl, Nl = P.tolist(), Nn.tolist()
    for i in range(n):
        nb = nbr[i].tolist()
        if len(nb) <= 1:
            continue
        incr = 100.0 / float(len(nb) - 1)
        row = [0.0] * 33
        for k in nb[1:]:
            f0, f1, f2, _ = pair_features(Pl[i], Nl[i], Pl[k], Nl[k])
            row[_bin11(11.0 * (f0 + M_PI) / (2.0 * M_PI))] += incr
            row[11 + _bin11(11.0 * (f1 + 1.0) * 0.5)] += incr
            row[22 + _bin11(11.0 * (f2 + 1.0) * 0.5)] += incr
        spfh[i] = row
    out = np.zeros((n, 33))
    sp = spfh.tolist()
    for i in range(n):
        nb = nbr[i].tolist()
        if len(nb) <= 1:
            continue
        dd = d2[i].tolist()
        acc = [0.0] * 33
        s = [0.0, 0.0, 0.0]
        for k, dist in zip(nb[1:], dd[1:]):
            if dist == 0.0:
                continue
            r = sp[k]
            for j in range(33):
                val = r[j] / dist
                s[j // 11] += val
                acc[j] += val
        for j in range(3):
            if s[j] != 0.0:
                s[j] = 100.0 / s[j]
        ri = sp[i]
        out[i] = [acc[j] * s[j // 11] + ri[j] for j in range(33)]
    return out


# ---------------------------------------------------------- feature matching ----
def feature_dist2(a, B):
    """nanoflann L2_Adaptor squared distance of a (33,) to every row of B."""
    D = a[None, :] - B
    Q = D * D
    r = np.zeros(len(B))
    for g in range(8):
        r = r + (((Q[:, 4 * g] + Q[:, 4 * g + 1]) + Q[:, 4 * g + 2]) + Q[:, 4 * g + 3])
    return r + Q[:, 32]


def feature_nn(A, B):
    """Nearest row of B (ties: lower index) for every row of A; -1 where no
    distance is below +inf.  A NaN distance never wins, as in nanoflann's
    search, whose candidates must compare `dist < worst` (np.argmin would
    return the first NaN)."""
    A = np.asarray(A, dtype=np.float64)
    B = np.asarray(B, dtype=np.float64)
    out = np.empty(len(A), dtype=np.int64)
    for i in range(len(A)):
        d = feature_dist2(A[i], B)
        d = np.where(np.isnan(d), np.inf, d)
        k = int(np.argmin(d)) if len(d) else -1  # argmin: first of equal minima
        out[i] = k if k >= 0 and d[k] < np.inf else -1
    return out


def correspondences_from_features(fs, ft, mutual_filter=True, mutual_consistent_ratio=0.1):
    """CorrespondencesFromFeatures -> int64 (K, 2) (source, target); a row
    without a nearest neighbour (NaN features) makes no pair."""
    ij = feature_nn(fs, ft)
    has = ij >= 0
    c0 = np.stack([np.arange(len(fs))[has], ij[has]], axis=1)
    if not mutual_filter:
        return c0
    ji = feature_nn(ft, fs)
    keep = ji[c0[:, 1]] == c0[:, 0]
    mutual = c0[keep]
    if len(mutual) >= int(np.float32(mutual_consistent_ratio) * np.float32(len(fs))):
        return mutual
    return c0


# ------------------------------------------------------------- 3x3 Jacobi SVD ----
_DBL_MIN = 2.2250738585072014e-308
_EPS2 = 2.0 * 2.220446049250313e-16
_SVD_SWEEPS = 64


def _rot_left(M, p, q, c, s):
    """applyOnTheLeft(p, q, J(c, s)): rows p, q."""
    for i in range(3):
        x, y = M[p][i], M[q][i]
        M[p][i] = c * x + s * y
        M[q][i] = -s * x + c * y


def _rot_right(M, p, q, c, s):
    """applyOnTheRight(p, q, J(c, s)) = rotation of columns p, q by J^T."""
    for i in range(3):
        x, y = M[i][p], M[i][q]
        M[i][p] = c * x - s * y
        M[i][q] = s * x + c * y


def _make_jacobi(x, y, z):
    deno = 2.0 * abs(y)
    if deno < _DBL_MIN:
        return 1.0, 0.0
    tau = (x - z) / deno
    w = math.sqrt(tau * tau + 1.0)
    t = 1.0 / (tau + w) if tau > 0.0 else 1.0 / (tau - w)
    sign_t = 1.0 if t > 0.0 else -1.0
    n = 1.0 / math.sqrt(t * t + 1.0)
    return n, -sign_t * (y / abs(y)) * abs(t) * n


def jacobi_svd3(A):
    """Eigen's JacobiSVD<Matrix3d>(A, ComputeFullU | ComputeFullV) -> (U, s, V)
    as nested lists; the two-sided Jacobi sweeps of real_2x2_jacobi_svd /
    makeJacobi, then |diagonal| descending (at most _SVD_SWEEPS sweeps)."""
    scale = max(abs(A[i][j]) for i in range(3) for j in range(3))
    if scale == 0.0:
        scale = 1.0
    W = [[A[i][j] / scale for j in range(3)] for i in range(3)]
    U = [[1.0 if i == j else 0.0 for j in range(3)] for i in range(3)]
    V = [[1.0 if i == j else 0.0 for j in range(3)] for i in range(3)]
    max_diag = max(abs(W[0][0]), abs(W[1][1]), abs(W[2][2]))
    for _ in range(_SVD_SWEEPS):
        finished = True
        for p in range(1, 3):
            for q in range(p):
                thr = max(_DBL_MIN, _EPS2 * max_diag)
                if abs(W[p][q]) > thr or abs(W[q][p]) > thr:
                    finished = False
                    # real_2x2_jacobi_svd on rows / cols (p, q)
                    m00, m01, m10, m11 = W[p][p], W[p][q], W[q][p], W[q][q]
                    t = m00 + m11
                    d = m10 - m01
                    if abs(d) < _DBL_MIN:
                        c1, s1 = 1.0, 0.0
                    else:
                        u = t / d
                        tmp = math.sqrt(1.0 + u * u)
                        s1 = 1.0 / tmp
                        c1 = u / tmp
                    # m.applyOnTheLeft(0, 1, rot1)
                    a00 = c1 * m00 + s1 * m10
                    a01 = c1 * m01 + s1 * m11
                    a11 = -s1 * m01 + c1 * m11
                    cr, sr = _make_jacobi(a00, a01, a11)
                    # j_left = rot1 * j_right^T; (c, s) * (c2, s2) = (c c2 - s s2, c s2 + s c2)
                    cl = c1 * cr - s1 * (-sr)
                    sl = c1 * (-sr) + s1 * cr
                    _rot_left(W, p, q, cl, sl)
                    _rot_right(U, p, q, cl, -sl)  # U.applyOnTheRight(p, q, j_left.transpose())
                    _rot_right(W, p, q, cr, sr)
                    _rot_right(V, p, q, cr, sr)
                    max_diag = max(max_diag, max(abs(W[p][p]), abs(W[q][q])))
        if finished:
            break
    s = [0.0, 0.0, 0.0]
    for i in range(3):
        a = W[i][i]
        s[i] = abs(a)
        if a < 0.0:
            for r in range(3):
                U[r][i] = -U[r][i]
    s = [v * scale for v in s]
    for i in range(3):
        pos = max(range(i, 3), key=lambda k: (s[k], -k))  # maxCoeff: the first maximum
        if s[pos] == 0.0:
            break
        if pos != i:
            s[i], s[pos] = s[pos], s[i]
            for r in range(3):
                U[r][i], U[r][pos] = U[r][pos], U[r][i]
                V[r][i], V[r][pos] = V[r][pos], V[r][i]
    return U, s, V


def _det3(M):
    return (M[0][0] * (M[1][1] * M[2][2] - M[2][1] * M[1][2])
            - M[1][0] * (M[0][1] * M[2][2] - M[2][1] * M[0][2])
            + M[2][0] * (M[0][1] * M[1][2] - M[1][1] * M[0][2]))


def umeyama3(src, dst):
    """Eigen::umeyama(src 3x3 columns = points, dst, with_scaling=false) of
    three point pairs (TransformationEstimationPointToPoint(False)) -> 4x4
    row-major nested list."""
    one_over_n = 1.0 / 3.0
    sm = [((src[0][k] + src[1][k]) + src[2][k]) * one_over_n for k in range(3)]
    dm = [((dst[0][k] + dst[1][k]) + dst[2][k]) * one_over_n for k in range(3)]
    sd = [[src[c][k] - sm[k] for k in range(3)] for c in range(3)]
    dd = [[dst[c][k] - dm[k] for k in range(3)] for c in range(3)]
    sigma = [[((dd[0][i] * sd[0][j] + dd[1][i] * sd[1][j]) + dd[2][i] * sd[2][j]) * one_over_n for j in range(3)]
             for i in range(3)]
    U, _, V = jacobi_svd3(sigma)
    S = [1.0, 1.0, 1.0]
    if _det3(U) * _det3(V) < 0.0:
        S[2] = -1.0
    R = [[((U[i][0] * S[0] * V[j][0] + U[i][1] * S[1] * V[j][1]) + U[i][2] * S[2] * V[j][2]) for j in range(3)]
         for i in range(3)]
    t = [dm[i] - ((R[i][0] * sm[0] + R[i][1] * sm[1]) + R[i][2] * sm[2]) for i in range(3)]
    return [R[0] + [t[0]], R[1] + [t[1]], R[2] + [t[2]], [0.0, 0.0, 0.0, 1.0]]


# ------------------------------------------------------------------ RANSAC ----
_MASK64 = (1 << 64) - 1


def draw(seed, n, corres_n):
    """The n-th random correspondence index: splitmix64 of seed + (n + 1) *
    golden, its high 32 bits scaled to [0, corres_n)."""
    z = (seed + (n + 1) * 0x9E3779B97F4A7C15) & _MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    z ^= z >> 31
    return ((z >> 32) * corres_n) >> 32


def _tp(T, p):
    return [((T[r][0] * p[0] + T[r][1] * p[1]) + T[r][2] * p[2]) + T[r][3] for r in range(3)]


def edge_length_ok(S, T, c, sim=0.9):
    """CorrespondenceCheckerBasedOnEdgeLength(sim).Check."""
    for i in range(3):
        for j in range(i + 1, 3):
            ds = _norm3([S[c[i][0]][k] - S[c[j][0]][k] for k in range(3)])
            dt = _norm3([T[c[i][1]][k] - T[c[j][1]][k] for k in range(3)])
            if ds < dt * sim or dt < ds * sim:
                return False
    return True


def distance_ok(S, T, c, M, thr):
    """CorrespondenceCheckerBasedOnDistance(thr).Check."""
    for cs, ct in c:
        q = _tp(M, S[cs])
        if _norm3([T[ct][k] - q[k] for k in range(3)]) > thr:
            return False
    return True


REG_BLOCK = 64


def validate(source, target, M, max_dist, tree):
    """GetRegistrationResultAndCorrespondences on the moved source ->
    (fitness, inlier_rmse, moved source)."""
    S = np.asarray(source, dtype=np.float64)
    Q = np.empty_like(S)
    for r in range(3):
        Q[:, r] = ((M[r][0] * S[:, 0] + M[r][1] * S[:, 1]) + M[r][2] * S[:, 2]) + M[r][3]
    Tg = tree.data
    r2 = max_dist * max_dist
    cand = tree.query_ball_point(Q, max_dist * (1.0 + 1e-9) + 1e-300)
    e2 = np.zeros(len(S))
    ok = np.zeros(len(S), dtype=bool)
    for i, c in enumerate(cand):
        if not c:
            continue
        c = np.asarray(c, dtype=np.int64)
        d = Q[i] - Tg[c]
        dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        dd = dd[dd < r2]
        if len(dd):
            ok[i] = True
            e2[i] = dd.min()
    n = len(S)
    nb = (n + REG_BLOCK - 1) // REG_BLOCK
    pad = np.zeros(nb * REG_BLOCK)
    pad[:n] = e2
    part = np.cumsum(pad.reshape(nb, REG_BLOCK), axis=1)[:, -1]
    err2 = 0.0
    for b in range(nb):
        err2 = err2 + float(part[b])
    cnt = int(ok.sum())
    if cnt == 0:
        return 0.0, 0.0, Q
    return cnt / n, math.sqrt(err2 / cnt), Q


def ransac_based_on_feature_matching(source, target, fs, ft, max_dist, seed=0, mutual_filter=True,
                                     edge_sim=0.9, max_iteration=100000, confidence=0.999):
    """registration_ransac_based_on_feature_matching (processing.py:98-111)
    -> dict(transformation, fitness, inlier_rmse, iterations, validations,
    corres)."""
    from scipy.spatial import cKDTree
    S = np.asarray(source, dtype=np.float64)
    Tg = np.asarray(target, dtype=np.float64)
    corres = correspondences_from_features(fs, ft, mutual_filter)
    best = {"transformation": np.eye(4), "fitness": 0.0, "inlier_rmse": 0.0, "iterations": 0, "validations": 0,
            "corres": corres}
    nc = len(corres)
    if nc < 3 or max_dist <= 0.0:
        return best
    tree = cKDTree(Tg)
    Sl, Tl = S.tolist(), Tg.tolist()
    cl = corres.tolist()
    est_k = max_iteration
    it = 0
    vals = 0
    thr2 = max_dist * max_dist
    log_conf = math.log(1.0 - confidence) if confidence < 1.0 else -math.inf
    while it < max_iteration and it < est_k:
        c = [cl[draw(seed, 3 * it + j, nc)] for j in range(3)]
        it += 1
        if not edge_length_ok(Sl, Tl, c, edge_sim):
            continue
        M = umeyama3([Sl[x[0]] for x in c], [Tl[x[1]] for x in c])
        if not distance_ok(Sl, Tl, c, M, max_dist):
            continue
        vals += 1
        fit, rmse, Q = validate(S, Tg, M, max_dist, tree)
        if fit > best["fitness"] or (fit == best["fitness"] and rmse < best["inlier_rmse"]):
            best.update(transformation=np.array(M), fitness=fit, inlier_rmse=rmse)
            d = Q[corres[:, 0]] - Tg[corres[:, 1]]
            dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
            ratio = float(np.count_nonzero(dd < thr2)) / float(nc)
            y = 1.0 - math.pow(ratio, 3.0)
            if y <= 0.0:
                est_d = 0.0
            else:
                den = math.log(y)
                est_d = log_conf / den if den != 0.0 else math.inf
            if est_d < est_k:
                est_k = int(math.ceil(est_d))
    best["iterations"] = it
    best["validations"] = vals
    return best
