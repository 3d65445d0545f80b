"""Global registration of merge_pro_360 on the GPU (processing.py:79-113):
radius search, FPFH features, feature matching and RANSAC bit for bit against
oracle/registration_oracle.py (Open3D's algorithms restated; parity with
Open3D itself is unpinned: not in this image, and its RANSAC draw is
unseeded), and the pose-free merge_pro_360 recovering a turntable's steps
(GPU only)."""
import math

import numpy as np
import pytest
import torch

from oracle import merge_oracle as mo
from oracle import registration_oracle as ro
from tests.test_registration_oracle import _rot, blob

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mg():
    from structured_light_for_3d_model_replication_amd import merge
    return merge


def _lists(idx, d2, cnt):
    idx, d2, cnt = idx.cpu().numpy(), d2.cpu().numpy(), cnt.cpu().numpy()
    return [idx[i, :cnt[i]] for i in range(len(cnt))], [d2[i, :cnt[i]] for i in range(len(cnt))]


def test_radius_search_vs_oracle(mg):
    """sorted (d2, index) lists, capped at max_nn, with duplicate points (ties
    broken by index) and a dense cluster whose queries overflow the LDS sort
    (more than 1024 candidates: the radix-select path)."""
    rng = np.random.default_rng(1)
    P = blob(3000, seed=2)
    P[100:140] = P[99]  # 41 identical points
    cluster = rng.normal(size=(1500, 3)) * 0.5 + np.array([0.0, 0.0, 30.0])
    P = np.concatenate([P, cluster])
    for radius, max_nn in ((6.0, 30), (3.0, 100), (12.0, 1024)):
        gi, gd = _lists(*mg.radius_search(P, radius, max_nn))
        wi, wd = ro.radius_neighbours(P, radius, max_nn)
        for i in range(len(P)):
            np.testing.assert_array_equal(gi[i], wi[i], err_msg=f"r={radius} point {i}")
            np.testing.assert_array_equal(gd[i], wd[i], err_msg=f"r={radius} point {i}")
    idx, d2, cnt = mg.radius_search(P, 0.0, 10)
    assert int(cnt.max()) == 0


def test_fpfh_vs_oracle(mg):
    """compute_fpfh_feature (radius 5 voxel, max_nn 100, processing.py:91-94)
    bit for bit, on a voxel-downsampled cloud with GPU normals (radius 2
    voxel, max_nn 30) as preprocess_point_cloud makes them; and a cloud with
    isolated points (no neighbours: zero features)."""
    vs = 3.0
    P = blob(6000, seed=3)
    Pd, _ = mg.voxel_down_sample(P, None, vs)
    Nd = mg.estimate_normals(Pd, 2 * vs, 30)
    got = mg.compute_fpfh_feature(Pd, Nd, 5 * vs, 100).cpu().numpy()
    want = ro.compute_fpfh(Pd.cpu().numpy(), Nd.cpu().numpy(), 5 * vs, 100)
    np.testing.assert_array_equal(got, want)
    Q = np.array([[0.0, 0, 0], [100.0, 0, 0], [100.5, 0, 0], [100.0, 0.5, 0.2]])
    NQ = np.array([[0.0, 0, 1], [0, 0, 1], [0, 1, 0], [1, 0, 0]])
    got = mg.compute_fpfh_feature(Q, NQ, 2.0, 100).cpu().numpy()
    np.testing.assert_array_equal(got, ro.compute_fpfh(Q, NQ, 2.0, 100))
    assert not got[0].any()


def test_feature_nn_vs_oracle(mg):
    rng = np.random.default_rng(4)
    A = rng.normal(size=(700, 33))
    B = np.concatenate([rng.normal(size=(900, 33)), A[:50]])
    np.testing.assert_array_equal(mg.feature_nn(A, B).cpu().numpy(), ro.feature_nn(A, B))
    B2 = np.concatenate([A[::-1], A[:5]])  # exact ties: the lower index
    np.testing.assert_array_equal(mg.feature_nn(A, B2).cpu().numpy(), np.arange(699, -1, -1))


def _reg_case(seed, n, ang, t, vs):
    P = blob(n, seed=seed)
    R = _rot(0.1, ang, -0.05)
    Q = P @ R.T + np.asarray(t)
    return P, Q, R


@pytest.mark.parametrize("case", [(7, 2500, 0.35, (12.0, 0.0, -5.0)), (9, 2000, -0.8, (-30.0, 8.0, 4.0))])
def test_ransac_vs_oracle(mg, case):
    """registration_ransac_based_on_feature_matching with the reference's
    settings (mutual filter, 1.5 voxel, edge 0.9, 100000 iterations, 0.999)
    on FPFH of two downsampled views of a rigid motion: transformation,
    fitness, RMSE, iterations, validations and correspondences equal to the
    oracle's run with the same seed; the motion recovered."""
    seed, n, ang, t = case
    vs = 2.5
    P, Q, R = _reg_case(seed, n, ang, t, vs)
    src, _ = mg.voxel_down_sample(P, None, vs)
    tgt, _ = mg.voxel_down_sample(Q, None, vs)
    sn, tn = mg.estimate_normals(src, 2 * vs, 30), mg.estimate_normals(tgt, 2 * vs, 30)
    sf, tf = mg.compute_fpfh_feature(src, sn, 5 * vs, 100), mg.compute_fpfh_feature(tgt, tn, 5 * vs, 100)
    got = mg.registration_ransac_based_on_feature_matching(src, tgt, sf, tf, True, 1.5 * vs, seed=seed)
    want = ro.ransac_based_on_feature_matching(src.cpu().numpy(), tgt.cpu().numpy(), sf.cpu().numpy(),
                                               tf.cpu().numpy(), 1.5 * vs, seed=seed)
    np.testing.assert_array_equal(got["transformation"], want["transformation"])
    assert got["fitness"] == want["fitness"] and got["inlier_rmse"] == want["inlier_rmse"]
    assert got["iterations"] == want["iterations"] and got["validations"] == want["validations"]
    assert got["correspondences"] == len(want["corres"])
    M = got["transformation"]
    ang_err = math.degrees(math.acos(min(1.0, (np.trace(M[:3, :3].T @ R) - 1.0) / 2.0)))
    assert ang_err < 3.0 and np.linalg.norm(M[:3, 3] - np.asarray(t)) < 3 * vs


def test_ransac_edges(mg):
    P = blob(200, seed=5)
    F = np.zeros((200, 33))
    r = mg.registration_ransac_based_on_feature_matching(P[:2], P[:2], F[:2], F[:2], True, 5.0)
    assert r["iterations"] == 0 and np.array_equal(r["transformation"], np.eye(4))
    r = mg.registration_ransac_based_on_feature_matching(np.zeros((0, 3)), P, np.zeros((0, 33)), F, True, 5.0)
    assert r["iterations"] == 0 and r["fitness"] == 0.0
    with pytest.raises(ValueError):
        mg.registration_ransac_based_on_feature_matching(P, P, F[:3], F, True, 5.0)


def test_merge_pro_360_pose_free_recovers_turntable(mg, tmp_path):
    """merge_pro_360(input_folder, output_path, voxel_size) with no poses, as
    the reference calls it: rendered turntable views 10 degrees apart
    (synth scene "turntable": a sphere with two bumps turning rigidly, no
    wall; structured-light decode + triangulation on the GPU), then FPFH +
    RANSAC + ICP per pair.  Every accumulated transform recovers the turntable
    motion within 1 degree and 2 mm."""
    from structured_light_for_3d_model_replication_amd import core, ply, synth
    rig = synth.Rig(H=240, W=320)
    cal = synth.make_calibration(rig)
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, rig.H, rig.W)
    degs = [0.0, 10.0, 20.0, 30.0]
    for i, deg in enumerate(degs):
        st, tex = synth.render_stack(rig, seed=300 + i, view_deg=deg, scene="turntable")
        res = eng.decode_triangulate(st.cuda(), texture=tex.cuda(), xyz_dtype=torch.float64)
        eng.sync()
        c = res["cloud"]
        n = c.total()
        ply.save_ply(c.xyz[:n].cpu().numpy(), c.bgr[:n].cpu().numpy(), str(tmp_path / f"scan_{i:03d}.ply"))
    vs = 3.0
    out = tmp_path / "merged.ply"
    P, C, N, Ts = mg.merge_pro_360(str(tmp_path), str(out), vs, return_transforms=True)
    assert out.exists() and P.shape[0] > 1000
    for i, deg in enumerate(degs):
        truth = mg.mat4(mg.rigid_inverse(synth.turntable_pose(degs[0])), synth.turntable_pose(deg))
        d = mg.mat4(mg.rigid_inverse(truth), Ts[i])
        ang = math.degrees(math.acos(min(1.0, (np.trace(d[:3, :3]) - 1.0) / 2.0)))
        assert ang < 1.0, f"view {i}: {ang:.3f} deg off"
        assert np.linalg.norm(d[:3, 3]) < 2.0, f"view {i}: {d[:3, 3]} mm off"


def test_mutual_matching_ties_and_nan_rows(mg):
    """The mutual filter's two directions (one pass over the pairs on the GPU)
    against the oracle's two scans: duplicated feature rows on both sides
    (ties to the lower index, in each direction), NaN rows (never a match),
    and a set just above / below the 0.1 mutual-pair fallback -- the
    correspondence counts of short RANSAC runs equal the oracle's."""
    rng = np.random.default_rng(11)
    P = blob(600, seed=12)
    Q = P + np.array([1.0, -2.0, 0.5])
    A = rng.integers(0, 4, size=(600, 33)).astype(np.float64)  # few distinct values: many exact ties
    B = np.concatenate([A[300:], A[:300]])
    B[5:9] = B[4]
    A[17] = np.nan
    B[40] = np.nan
    for a_f, b_f in ((A, B), (A, rng.normal(size=(600, 33)))):
        got = mg.registration_ransac_based_on_feature_matching(P, Q, a_f, b_f, True, 1.0, max_iteration=5, seed=3)
        want = ro.correspondences_from_features(a_f, b_f, True)
        assert got["correspondences"] == len(want)
