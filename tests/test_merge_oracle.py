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
