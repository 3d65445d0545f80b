"""Merge-stage oracle (oracle/merge_oracle.py) on CPU: hand-checked voxel cases
and the brute-force kNN means against scipy's cKDTree.  Parity with Open3D
itself is unpinned (Open3D is not installed)."""
import numpy as np
import pytest

from oracle import merge_oracle as mo


def test_voxel_grid_origin_and_order():
    # grid origin min - vs/2: 0 and 0.05 fall in different voxels at vs = 0.1
    P = np.array([[1, 1, 1], [0, 0, 0], [0.05, 0, 0], [1.04, 1, 1], [5, 5, 5]], float)
    C = np.array([[10, 20, 30], [0, 0, 0], [255, 255, 255], [11, 21, 31], [1, 2, 3]], np.uint8)
    Q, Cq = mo.voxel_down_sample(P, C, 0.1)
    np.testing.assert_array_equal(Q, [[0, 0, 0], [0.05, 0, 0], [(1 + 1.04) / 2, 1, 1], [5, 5, 5]])
    # colour means as Open3D holds them (c/255), written round-half-away
    avg = (np.array([10, 20, 30]) / 255.0 + np.array([11, 21, 31]) / 255.0) / 2
    np.testing.assert_array_equal(Cq[2], np.floor(avg * 255.0 + 0.5).astype(np.uint8))
    with pytest.raises(ValueError):
        mo.voxel_down_sample(P, C, 0.0)
    with pytest.raises(ValueError):
        mo.voxel_down_sample(np.array([[0, 0, 0], [1e9, 0, 0]], float), None, 1e-3)


def test_voxel_sums_in_point_order():
    rng = np.random.default_rng(1)
    P = rng.normal(0, 1, (2000, 3)) * 1e3
    Q, _ = mo.voxel_down_sample(P, None, 250.0)
    lo = P.min(0) - 125.0
    key = [tuple(np.floor((p - lo) / 250.0).astype(int)) for p in P]
    ref = {}
    for p, k in zip(P, key):
        s, n = ref.get(k, (np.zeros(3), 0))
        ref[k] = (s + p, n + 1)  # sequential, in index order
    exp = np.array([ref[k][0] / ref[k][1] for k in sorted(ref)])
    np.testing.assert_array_equal(Q, exp)


def test_knn_means_against_ckdtree():
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(2)
    P = np.concatenate([rng.normal(0, 1, (1500, 3)), rng.uniform(-8, 8, (40, 3))])
    avg = mo.knn_mean_distances(P, 20)
    d, _ = cKDTree(P).query(P, k=20)
    np.testing.assert_allclose(avg, d.mean(1), rtol=1e-14)
    ind = mo.statistical_outlier_indices(avg, 2.0)
    assert 0 < len(ind) < len(P)
    # the far uniform points are the ones removed
    assert np.mean(ind >= 1500) < 0.5


def test_statistical_edge_cases():
    assert len(mo.statistical_outlier_indices(np.zeros(0), 2.0)) == 0
    # all points coincide: every mean is 0, nothing kept (0 < mean fails)
    ind, avg = mo.remove_statistical_outlier(np.ones((30, 3)), 20, 2.0)
    assert len(ind) == 0 and np.all(avg == 0)
    # a single point: std over n - 1 = 0 points is nan -> nothing kept
    ind, _ = mo.remove_statistical_outlier(np.array([[1.0, 2.0, 3.0]]), 20, 2.0)
    assert len(ind) == 0


def test_det_math_within_one_ulp():
    """The fdlibm acos / cos both normal paths use (oracle and slmerge.hip)
    stay within 1 ulp of the exact value on FastEigen3x3's ranges (acos on
    [-1, 1], cos on [0, pi/3] and [2pi/3, pi])."""
    import mpmath
    mpmath.mp.prec = 120
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.uniform(-1, 1, 400), [-1.0, 1.0, 0.5, -0.5, 0.0, 1 - 2**-53, -1 + 2**-53]])
    for x in xs:
        e = float(mpmath.acos(mpmath.mpf(float(x))))
        assert abs(mo.acos_det(float(x)) - e) <= np.spacing(abs(e)) if e else mo.acos_det(float(x)) == 0.0
    ys = np.concatenate([rng.uniform(0, np.pi / 3, 300), rng.uniform(2 * np.pi / 3, np.pi, 300),
                         [0.0, np.pi / 3, 2.09439510239319549, np.pi]])
    for y in ys:
        e = float(mpmath.cos(mpmath.mpf(float(y))))
        assert abs(mo.cos_det(float(y)) - e) <= np.spacing(abs(e))


def test_normals_oracle_is_the_smallest_eigenvector():
    """estimate_normals' FastEigen3x3 vs numpy's eigh of the same neighbour
    covariance: the same direction (|cos| = 1 within 1e-12) wherever the
    smallest eigenvalue is well separated; unit length everywhere."""
    rng = np.random.default_rng(4)
    u = rng.normal(size=(1500, 3))
    P = 50.0 * u / np.linalg.norm(u, axis=1, keepdims=True) + rng.normal(0, 0.3, (1500, 3))
    N = mo.estimate_normals(P, 9.0, 30)
    np.testing.assert_allclose(np.linalg.norm(N, axis=1), 1.0, rtol=1e-12)
    checked = 0
    for i, nb in enumerate(mo.hybrid_neighbours(P, 9.0, 30)):
        if len(nb) < 3:
            continue
        w, v = np.linalg.eigh(np.cov(P[nb].T, bias=True))
        if w[1] - w[0] > 1e-6 * w[2]:
            assert abs(abs(v[:, 0] @ N[i]) - 1.0) < 1e-9
            checked += 1
    assert checked > 1000


def test_normals_oracle_degenerate_cases():
    # fewer than 3 neighbours -> identity covariance -> (0, 0, 1); a plane -> +-z
    np.testing.assert_array_equal(mo.estimate_normals(np.array([[0.0, 0, 0], [1.0, 0, 0]]), 0.5),
                                  [[0, 0, 1.0], [0, 0, 1.0]])
    g = np.arange(6, dtype=float)
    plane = np.stack(np.meshgrid(g, g, [0.0], indexing="ij"), -1).reshape(-1, 3)
    N = mo.estimate_normals(plane, 1.5, 30)
    np.testing.assert_array_equal(np.abs(N), np.tile([0.0, 0.0, 1.0], (len(plane), 1)))


def _sheet(n_side=90, seed=0):
    """A bumpy height field (a surface with structure in every direction)."""
    rng = np.random.default_rng(seed)
    u, v = np.meshgrid(np.linspace(-60, 60, n_side), np.linspace(-60, 60, n_side))
    u = u.ravel() + rng.uniform(-0.3, 0.3, u.size)
    v = v.ravel() + rng.uniform(-0.3, 0.3, v.size)
    z = 8 * np.sin(u / 13.0) * np.cos(v / 17.0) + 0.004 * u * v
    return np.stack([u, v, z], 1)


def _motion(deg, t):
    a = np.radians(deg)
    R = np.array([[np.cos(a), -np.sin(a), 0.0], [np.sin(a), np.cos(a), 0.0], [0.0, 0.0, 1.0]])
    b = np.radians(deg / 2)
    R = R @ np.array([[1.0, 0.0, 0.0], [0.0, np.cos(b), -np.sin(b)], [0.0, np.sin(b), np.cos(b)]])
    M = np.eye(4)
    M[:3, :3] = R
    M[:3, 3] = t
    return M


def test_icp_oracle_recovers_a_rigid_motion():
    """The point-to-plane ICP restatement (processing.py:154-156) converges to
    a known small motion from the identity: target = M(source)."""
    from oracle import merge_oracle as m
    S = _sheet()
    M = _motion(1.5, [0.8, -0.5, 0.6])
    T = m._transform(S, M)
    N = m.estimate_normals(T, 6.0, 30)
    r = m.registration_icp_point_to_plane(S, T, N, 5.0, None, max_iteration=60)
    np.testing.assert_allclose(r["transformation"], M, atol=1e-6)
    assert r["fitness"] == 1.0 and r["inlier_rmse"] < 1e-6 and 0 < r["iterations"] < 60


def test_rigid_inverse_and_mat4():
    from oracle import merge_oracle as m
    M = _motion(33.0, [10.0, -20.0, 5.0])
    I = np.array(m.mat4(m.rigid_inverse(M).tolist(), M.tolist()))
    np.testing.assert_allclose(I, np.eye(4), atol=1e-12)
    U = m.icp_update([0.0] * 29)  # singular system: the identity update
    assert np.array_equal(np.array(U), np.eye(4))
