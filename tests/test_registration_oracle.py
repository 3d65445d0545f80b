"""The global-registration oracle (oracle/registration_oracle.py) on its own,
CPU only: the fdlibm atan2 against libm, the 3x3 Jacobi SVD against LAPACK,
Umeyama on exact rigid motions, FPFH's invariance under rigid motion, the
feature matching and RANSAC recovering a known motion.  (Parity with Open3D is
unpinned: it is not in this image.)"""
import math

import numpy as np

from oracle import merge_oracle as mo
from oracle import registration_oracle as ro


def _rot(ax, ay, az):
    cx, sx, cy, sy, cz, sz = math.cos(ax), math.sin(ax), math.cos(ay), math.sin(ay), math.cos(az), math.sin(az)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def blob(n, seed=0):
    """An asymmetric closed surface (a lumpy ellipsoid) sampled at n points."""
    rng = np.random.default_rng(seed)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    r = 40.0 * (1.0 + 0.25 * np.sin(3.0 * u[:, 0]) * np.cos(2.0 * u[:, 1]) + 0.15 * u[:, 2] ** 3)
    return u * r[:, None] * np.array([1.0, 0.8, 0.6])


def test_atan2_within_one_ulp_of_libm():
    rng = np.random.default_rng(1)
    for _ in range(20000):
        y, x = rng.normal(size=2) * 10.0 ** rng.uniform(-6, 6, size=2)
        a, b = ro.atan2_det(y, x), math.atan2(y, x)
        assert abs(a - b) <= math.ulp(b), (y, x)
    for y, x in [(0.0, -1.0), (-0.0, -1.0), (1.0, 0.0), (-1.0, 0.0), (0.0, 0.0), (-0.0, 0.0), (1.0, 1.0),
                 (1e-300, -1.0), (1e300, 1e-300), (-2.0, 1.0)]:
        assert ro.atan2_det(y, x) == math.atan2(y, x), (y, x)


def test_jacobi_svd3_against_lapack():
    rng = np.random.default_rng(2)
    for k in range(300):
        A = rng.normal(size=(3, 3)) * 10.0 ** rng.uniform(-3, 3)
        if k % 7 == 0:
            A[:, 2] = A[:, 0] + A[:, 1]  # rank 2
        U, s, V = ro.jacobi_svd3(A.tolist())
        U, V, s = np.array(U), np.array(V), np.array(s)
        ref = np.linalg.svd(A, compute_uv=False)
        np.testing.assert_allclose(s, ref, rtol=1e-12, atol=1e-12 * ref[0])
        np.testing.assert_allclose(U @ np.diag(s) @ V.T, A, atol=1e-12 * ref[0])
        np.testing.assert_allclose(U.T @ U, np.eye(3), atol=1e-13)
        np.testing.assert_allclose(V.T @ V, np.eye(3), atol=1e-13)
    U, s, V = ro.jacobi_svd3([[0.0] * 3] * 3)
    assert s == [0.0, 0.0, 0.0] and U == [[1.0, 0, 0], [0, 1.0, 0], [0, 0, 1.0]]


def test_umeyama_recovers_rigid_motion():
    rng = np.random.default_rng(3)
    for _ in range(200):
        R = _rot(*rng.uniform(-math.pi, math.pi, size=3))
        t = rng.normal(size=3) * 50
        S = rng.normal(size=(3, 3)) * 30
        D = S @ R.T + t
        M = np.array(ro.umeyama3(S.tolist(), D.tolist()))
        np.testing.assert_allclose(M[:3, :3], R, atol=1e-9)
        np.testing.assert_allclose(M[:3, 3], t, atol=1e-7)
        assert np.linalg.det(M[:3, :3]) > 0


def test_radius_neighbours_sorted_and_capped():
    P = blob(400, seed=4)
    idx, d2 = ro.radius_neighbours(P, 12.0, 10)
    for i in range(len(P)):
        assert idx[i][0] == i and d2[i][0] == 0.0  # itself first
        assert len(idx[i]) <= 10
        assert np.all(np.diff(d2[i]) >= 0)
        assert np.all(d2[i] < 144.0)


def test_fpfh_invariant_under_rigid_motion():
    P = blob(900, seed=5)
    N = mo.estimate_normals(P, 8.0, 30)
    F = ro.compute_fpfh(P, N, 20.0, 100)
    R = _rot(0.3, -0.2, 0.5)
    Q = P @ R.T + np.array([10.0, -4.0, 7.0])
    NQ = N @ R.T  # the same normals moved (estimate_normals' eigenvector signs are arbitrary)
    FQ = ro.compute_fpfh(Q, NQ, 20.0, 100)
    assert F.shape == (900, 33)
    np.testing.assert_allclose(F.sum(axis=1), FQ.sum(axis=1), rtol=1e-6, atol=1e-6)
    for k in range(3):  # every third sums to 200 (the SPFH's 100 plus the weighted neighbours' 100)
        np.testing.assert_allclose(F[:, 11 * k:11 * k + 11].sum(axis=1), 200.0, rtol=1e-9)
    assert np.mean(np.abs(F - FQ)) < 1.0  # rounding can move a pair across a bin edge, rarely


def test_feature_nn_order_and_ties():
    rng = np.random.default_rng(6)
    A = rng.normal(size=(50, 33))
    B = np.concatenate([A[::-1], A[:5]])  # duplicates: ties to the lower index
    nn = ro.feature_nn(A, B)
    np.testing.assert_array_equal(nn, np.arange(49, -1, -1))
    d = ro.feature_dist2(A[0], B)
    assert d[49] == 0.0 and d[50] == 0.0 and nn[0] == 49


def test_ransac_recovers_motion():
    P = blob(800, seed=7)
    N = mo.estimate_normals(P, 8.0, 30)
    F = ro.compute_fpfh(P, N, 20.0, 100)
    R = _rot(0.0, 0.35, 0.0)
    t = np.array([12.0, 0.0, -5.0])
    Q = P @ R.T + t
    NQ = mo.estimate_normals(Q, 8.0, 30)
    FQ = ro.compute_fpfh(Q, NQ, 20.0, 100)
    res = ro.ransac_based_on_feature_matching(P, Q, F, FQ, 6.0, seed=11)
    M = res["transformation"]
    assert res["fitness"] > 0.9 and res["validations"] >= 1 and res["iterations"] >= 1
    np.testing.assert_allclose(M[:3, :3], R, atol=1e-6)
    np.testing.assert_allclose(M[:3, 3], t, atol=1e-4)
    # the same seed: the same run; another seed may stop elsewhere but is just as good
    res2 = ro.ransac_based_on_feature_matching(P, Q, F, FQ, 6.0, seed=11)
    assert res2["iterations"] == res["iterations"] and np.array_equal(res2["transformation"], M)


def test_ransac_degenerate_inputs():
    P = blob(50, seed=8)
    F = np.zeros((50, 33))
    res = ro.ransac_based_on_feature_matching(P[:2], P[:2], F[:2], F[:2], 5.0)
    assert res["iterations"] == 0 and np.array_equal(res["transformation"], np.eye(4))
    res = ro.ransac_based_on_feature_matching(P, P, F, F, 0.0)  # max_correspondence_distance <= 0
    assert res["iterations"] == 0 and np.array_equal(res["transformation"], np.eye(4))
    # all features equal: every source point matches target 0, one-way (no mutual pairs beyond one)
    c = ro.correspondences_from_features(F, F, True)
    np.testing.assert_array_equal(c[:, 1], 0)
