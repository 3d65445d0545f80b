"""HIP path vs the CPU oracle and the reference's golden fixtures (GPU only).

Bar: col/row maps, masks, point set and order bit-exact; XYZ bit-exact in the
f64 output mode and equal to the round-to-nearest float32 of the reference's
f64 in the f32 mode (|rel err| <= 2**-24, far inside the 1e-4 tolerance of
BASELINE.json).
"""
import numpy as np
import pytest
import torch

from oracle import sl_oracle as o
from tests import golden_io as g

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from structured_light_for_3d_model_replication_amd import core
    return core.Reconstructor(torch.device("cuda", 0))


def _run(eng, stack, tex, calib, n_cols, n_rows, mask_mode="adaptive", xyz_dtype=torch.float64, maps=True,
         poses=None):
    st = torch.as_tensor(np.ascontiguousarray(stack)).cuda()
    H, W = st.shape[-2:]
    eng.set_calibration(calib, H, W)
    tx = None if tex is None else torch.as_tensor(np.ascontiguousarray(tex)).cuda()
    res = eng.decode_triangulate(st, n_cols, n_rows, texture=tx, mask_mode=mask_mode, maps=maps, cloud=True,
                                 xyz_dtype=xyz_dtype, poses=poses)
    eng.sync()
    return res


def _cloud_np(cloud):
    off = cloud.offsets()
    return cloud.xyz[: off[-1]].cpu().numpy(), cloud.bgr[: off[-1]].cpu().numpy(), off


def _assert_f32(xyz32, P):
    assert xyz32.dtype == np.float32
    np.testing.assert_array_equal(xyz32, P.astype(np.float32))
    if len(P):
        rel = np.abs(xyz32.astype(np.float64) - P) / np.maximum(np.abs(P), 1e-30)
        assert rel.max() <= 2.0 ** -24


def _assert_fast(xyz32, P):
    """SL_XYZ_F32_FAST's bound: per coordinate |rel err| <= (11 + 10*16) 2^-24
    ~ 1.02e-5 of the reference's f64 (BASELINE tolerance 1e-4)."""
    assert xyz32.dtype == np.float32
    err = np.abs(xyz32.astype(np.float64) - P)
    assert np.all(err <= 171 * 2.0 ** -24 * np.abs(P) + 1e-30)


STACK_CASES = g.names(func={"sl", "mp", "generate_cloud"})


@pytest.mark.parametrize("name", STACK_CASES)
def test_golden_fused(eng, name):
    d = g.load(name)
    m = d["meta"]
    res = _run(eng, d["stack"], d["texture"], d["calib"], m["n_cols"], m["n_rows"], m["mask_mode"])
    np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), d["col_map"])
    np.testing.assert_array_equal(res["row_map"][0].cpu().numpy(), d["row_map"])
    np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), d["mask"])
    xyz, bgr, off = _cloud_np(res["cloud"])
    assert off[-1] == len(d["P"])
    np.testing.assert_array_equal(xyz.view(np.uint64), d["P"].view(np.uint64))
    np.testing.assert_array_equal(bgr, d["C"])


@pytest.mark.parametrize("name", STACK_CASES)
def test_golden_cloud_only_f32(eng, name):
    d = g.load(name)
    m = d["meta"]
    res = _run(eng, d["stack"], d["texture"], d["calib"], m["n_cols"], m["n_rows"], m["mask_mode"],
               xyz_dtype=torch.float32, maps=False)
    xyz, bgr, off = _cloud_np(res["cloud"])
    assert off[-1] == len(d["P"])
    _assert_f32(xyz, d["P"])
    np.testing.assert_array_equal(bgr, d["C"])


def test_golden_reconstruct_only(eng):
    d = g.load("sl_reconstruct_colour_clip")
    H, W = d["col_map"].shape
    eng.set_calibration(d["calib"], H, W)
    for dt in (torch.float64, torch.float32):
        cloud = eng.triangulate_maps(torch.from_numpy(d["col_map"]), torch.from_numpy(d["mask"]),
                                     torch.from_numpy(d["texture"]), xyz_dtype=dt)
        eng.sync()
        xyz, bgr, off = _cloud_np(cloud)
        assert off[-1] == len(d["P"])
        if dt == torch.float64:
            np.testing.assert_array_equal(xyz.view(np.uint64), d["P"].view(np.uint64))
        else:
            _assert_f32(xyz, d["P"])
        np.testing.assert_array_equal(bgr, d["C"])


def test_golden_threshold_pins(eng):
    d = g.load("adaptive_threshold_pins")
    for k in range(d["meta"]["n"]):
        w, b = d[f"white_{k}"], d[f"black_{k}"]
        st = torch.from_numpy(np.stack([w, b, w, b])).cuda()
        res = eng.decode_triangulate(st, 2, 2, maps=True, cloud=False)
        eng.sync()
        np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), d[f"mask_{k}"])
        nf, dr, _, _ = eng.last_thresholds(0)
        assert nf.view(np.uint32) == d[f"nf_{k}"].view(np.uint32)
        assert dr == np.max(w.astype(np.float32) - b.astype(np.float32))


def test_golden_errors(eng):
    d = g.load("errors")
    n_img = {"three": 3, "odd9": 9, "odd15": 15}
    for tag, exc in d["meta"]["errors"].items():
        st = torch.from_numpy(np.ascontiguousarray(d["stack"][: n_img[tag]])).cuda()
        with pytest.raises({"ValueError": ValueError, "IndexError": IndexError}[exc]):
            eng.decode_triangulate(st, 16, 8, maps=True, cloud=False)


# ------------------------------------------------ synthetic, oracle-checked ----

@pytest.mark.parametrize("W", [160, 150])
def test_truncated_stacks_vs_oracle(eng, W):
    """Stacks with fewer (pattern, inverse) pairs than code bits
    (sl_system.py:553-570 stops at the last image): 3 / 8 / 9 column pairs
    (codes shifted up with the lowest binary bit repeated below), all 11
    columns and 4 of 11 rows, and every pair -- the byte-lane Gray conversion's
    A-only, A+B and shifted cases -- bit for bit against the oracle, on the
    vector path (W % 16 == 0) and the byte path."""
    rig, st, tex, cal = _render(96, W, 1920, 1080, seed=7 + W, rows=True)
    sth, texh = st.cpu().numpy(), tex.cpu().numpy()
    # (+ n_cols 65536: 16-bit column codes, 8 of them in the second byte lane;
    # n_cols 16 / n_rows 8: 4- and 3-bit codes)
    for k, nco, nro in ((3, 1920, 1080), (8, 1920, 1080), (9, 1920, 1080), (11, 1920, 1080), (15, 1920, 1080),
                        (22, 1920, 1080), (22, 65536, 1080), (22, 16, 8)):
        n = 2 + 2 * k
        col, row, mask, P, C = o.decode_triangulate(list(sth[:n]), texh, cal, nco, nro, "adaptive")
        res = _run(eng, sth[:n], texh, cal, nco, nro, xyz_dtype=torch.float64, maps=True)
        tag = f"{k} pairs, {nco} x {nro}"
        np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col, err_msg=tag)
        np.testing.assert_array_equal(res["row_map"][0].cpu().numpy(), row, err_msg=tag)
        np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask, err_msg=tag)
        xyz, bgr, off = _cloud_np(res["cloud"])
        assert off[-1] == len(P), tag
        np.testing.assert_array_equal(xyz.view(np.uint64), P.view(np.uint64))
        np.testing.assert_array_equal(bgr, C)


def _render(H, W, Wp, Hp, seed, rows=True, view=0.0, device="cuda"):
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.Rig(H=H, W=W, Wp=Wp, Hp=Hp)
    st, tex = synth.render_stack(rig, seed=seed, include_rows=rows, view_deg=view, device=device)
    return rig, st, tex, synth.make_calibration(rig)


@pytest.mark.parametrize("H,W,Wp,Hp,n_cols,n_rows,rows,mode", [
    (720, 1280, 1024, 768, 1024, 768, False, "adaptive"),     # config 1 shape
    (1080, 1920, 1920, 1080, 1920, 1080, True, "adaptive"),   # config 3 view
    (1080, 1920, 1920, 1080, 1920, 1080, True, "fixed"),
    (300, 400, 1280, 800, 1280, 800, True, "adaptive"),       # 11+10 bits: generic kernel
    (250, 333, 1920, 1080, 1920, 1080, True, "adaptive"),     # HW % 16 != 0: byte path
])
def test_synthetic_vs_oracle(eng, H, W, Wp, Hp, n_cols, n_rows, rows, mode):
    rig, st, tex, cal = _render(H, W, Wp, Hp, seed=H + W, rows=rows)
    sth, texh = st.cpu().numpy(), tex.cpu().numpy()
    col, row, mask, P, C = o.decode_triangulate(list(sth), texh, cal, n_cols, n_rows, mode)
    for maps in (True, False):
        for dt in (torch.float32, torch.float64):
            res = _run(eng, sth, texh, cal, n_cols, n_rows, mode, xyz_dtype=dt, maps=maps)
            if maps:
                np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
                np.testing.assert_array_equal(res["row_map"][0].cpu().numpy(), row)
                np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask)
            xyz, bgr, off = _cloud_np(res["cloud"])
            assert off[-1] == len(P)
            if dt == torch.float64:
                np.testing.assert_array_equal(xyz.view(np.uint64), P.view(np.uint64))
            else:
                _assert_f32(xyz, P)
            np.testing.assert_array_equal(bgr, C)


@pytest.mark.parametrize("H,W,Wp,Hp,n_cols,n_rows,rows", [
    (720, 1280, 1024, 768, 1024, 768, False),     # config 1 (specialised maps-only kernel)
    (1080, 1920, 1920, 1080, 1920, 1080, True),   # 11+11 bits (specialised maps-only kernel)
    (300, 400, 1280, 800, 1280, 800, True),       # generic kernel
])
def test_maps_only_vs_oracle(eng, H, W, Wp, Hp, n_cols, n_rows, rows):
    """gray_decode's device call (maps, no cloud), which runs its own k_decode
    instantiations: col/row maps and mask bit-exact vs the oracle."""
    rig, st, tex, cal = _render(H, W, Wp, Hp, seed=H + 7, rows=rows)
    sth = st.cpu().numpy()
    col, row, mask = o.gray_decode_images(list(sth), n_cols, n_rows, o.MASK_ADAPTIVE)
    res = eng.decode_triangulate(st, n_cols, n_rows, maps=True, cloud=False)
    eng.sync()
    np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
    np.testing.assert_array_equal(res["row_map"][0].cpu().numpy(), row)
    np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask)


def test_maps_only_fresh_context_no_calibration():
    """gray_decode on a context that was never calibrated (Old/process_cloud.py
    main: gray_decode before the calibration is loaded) at the CLI's 1920x1080
    capture size: k_decode loads no calibration table on a maps-only call."""
    from structured_light_for_3d_model_replication_amd import core
    rig, st, tex, cal = _render(1080, 1920, 1920, 1080, seed=11)
    fresh = core.Reconstructor(torch.device("cuda", 0))
    try:
        col, row, mask = o.gray_decode_images(list(st.cpu().numpy()), 1920, 1080, o.MASK_ADAPTIVE)
        for mode, m in (("adaptive", mask), ("fixed", None)):
            res = fresh.decode_triangulate(st, 1920, 1080, maps=True, cloud=False, mask_mode=mode)
            fresh.sync()
            np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
            np.testing.assert_array_equal(res["row_map"][0].cpu().numpy(), row)
            if m is None:
                m = o.gray_decode_images(list(st.cpu().numpy()), 1920, 1080, o.MASK_FIXED)[2]
            np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), m)
    finally:
        fresh.close()


def test_maps_only_after_wide_or_mismatched_calibration():
    """Maps-only calls on a context calibrated for a wider projector (Wp =
    3840 > the decode's LDS plane table) or for another frame size: the maps
    and mask stay bit-exact (no table is read), and a cloud call afterwards on
    the matching frame is still exact."""
    from structured_light_for_3d_model_replication_amd import core, synth
    fresh = core.Reconstructor(torch.device("cuda", 0))
    try:
        wide = synth.Rig(H=540, W=960, Wp=3840, Hp=2160)
        fresh.set_calibration(synth.make_calibration(wide), wide.H, wide.W)
        for H, W in ((1080, 1920), (540, 960)):
            rig, st, tex, cal = _render(H, W, 1920, 1080, seed=H + 3)
            col, row, mask = o.gray_decode_images(list(st.cpu().numpy()), 1920, 1080, o.MASK_ADAPTIVE)
            res = fresh.decode_triangulate(st, 1920, 1080, maps=True, cloud=False)
            fresh.sync()
            np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
            np.testing.assert_array_equal(res["row_map"][0].cpu().numpy(), row)
            np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask)
        # a cloud with the wide calibration (Wp > 2048: the three-kernel path)
        rig, st, tex, _ = _render(540, 960, 1920, 1080, seed=77)
        cal = synth.make_calibration(wide)
        sth, texh = st.cpu().numpy(), tex.cpu().numpy()
        _, _, _, P, C = o.decode_triangulate(list(sth), texh, cal, 1920, 1080)
        res = _run(fresh, sth, texh, cal, 1920, 1080, xyz_dtype=torch.float64)
        xyz, bgr, off = _cloud_np(res["cloud"])
        assert off[-1] == len(P)
        np.testing.assert_array_equal(xyz.view(np.uint64), P.view(np.uint64))
        np.testing.assert_array_equal(bgr, C)
    finally:
        fresh.close()


def test_full_4k_view_vs_oracle(eng):
    """Config 2 (3840x2160, 11+11 bits) at full size, bit-exact vs the oracle."""
    rig, st, tex, cal = _render(2160, 3840, 1920, 1080, seed=2)
    sth, texh = st.cpu().numpy(), tex.cpu().numpy()
    col, row, mask, P, C = o.decode_triangulate(list(sth), texh, cal, 1920, 1080)
    res = _run(eng, sth, texh, cal, 1920, 1080, xyz_dtype=torch.float32)
    np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
    np.testing.assert_array_equal(res["row_map"][0].cpu().numpy(), row)
    np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask)
    xyz, bgr, off = _cloud_np(res["cloud"])
    assert off[-1] == len(P)
    _assert_f32(xyz, P)
    np.testing.assert_array_equal(bgr, C)


def test_multiview_batch_offsets_and_pose(eng):
    """Several views in one launch: merged order = view order, per-view offsets,
    turntable pose epilogue (f64, oracle.apply_pose order)."""
    from structured_light_for_3d_model_replication_amd import synth
    V, H, W = 4, 240, 320
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    stacks, texes = [], []
    for v in range(V):
        s, t = synth.render_stack(rig, seed=50 + v, view_deg=10.0 * v)
        stacks.append(s.numpy())
        texes.append(t.numpy())
    poses = np.stack([synth.turntable_pose(10.0 * v) for v in range(V)])
    eng.set_calibration(cal, H, W)
    res = eng.decode_triangulate(torch.from_numpy(np.stack(stacks)).cuda(), texture=torch.from_numpy(
        np.stack(texes)).cuda(), maps=True, cloud=True, xyz_dtype=torch.float64,
        poses=torch.from_numpy(poses).cuda())
    eng.sync()
    xyz, bgr, off = _cloud_np(res["cloud"])
    start = 0
    for v in range(V):
        col, row, mask, P, C = o.decode_triangulate(list(stacks[v]), texes[v], cal, pose=poses[v])
        assert off[v] == start and off[v + 1] - off[v] == len(P)
        np.testing.assert_array_equal(xyz[off[v]:off[v + 1]].view(np.uint64), P.view(np.uint64))
        np.testing.assert_array_equal(bgr[off[v]:off[v + 1]], C)
        np.testing.assert_array_equal(res["col_map"][v].cpu().numpy(), col)
        np.testing.assert_array_equal(res["mask"][v].cpu().numpy(), mask)
        start += len(P)


def test_non_pinhole_nc(eng):
    """A calib whose Nc is not the pinhole rays of cam_K: rays come from Nc
    (sl_system.py:605-606), uploaded and read per pixel."""
    rig, st, tex, cal = _render(120, 160, 1920, 1080, seed=77)
    cal = dict(cal)
    rng = np.random.default_rng(0)
    Nc = cal["Nc"] * (1.0 + 1e-3 * rng.standard_normal(cal["Nc"].shape))
    cal["Nc"] = Nc
    sth, texh = st.cpu().numpy(), tex.cpu().numpy()
    col, row, mask, P, C = o.decode_triangulate(list(sth), texh, cal)
    for maps in (True, False):  # maps + cloud and cloud-only kernels of the Nc path
        res = _run(eng, sth, texh, cal, 1920, 1080, maps=maps)
        xyz, bgr, off = _cloud_np(res["cloud"])
        assert off[-1] == len(P)
        np.testing.assert_array_equal(xyz.view(np.uint64), P.view(np.uint64))
        np.testing.assert_array_equal(bgr, C)
        if maps:
            np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
            np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask)


def test_repeat_calls_are_stable(eng):
    """Back-to-back calls on one context (state reset by k_stats) give the
    same answer; white-as-texture path (texture=None)."""
    rig, st, tex, cal = _render(480, 640, 1920, 1080, seed=9)
    sth = st.cpu().numpy()
    col, row, mask, P, C = o.decode_triangulate(list(sth), None, cal)
    for _ in range(3):
        res = _run(eng, sth, None, cal, 1920, 1080, xyz_dtype=torch.float32)
        xyz, bgr, off = _cloud_np(res["cloud"])
        assert off[-1] == len(P)
        _assert_f32(xyz, P)
        np.testing.assert_array_equal(bgr, C)


def test_launch_groups_and_view_offsets(eng):
    """A batch larger than one launch group (64K chunks): 33 views of
    1920x1080 are 66825 chunks -> two groups (32 + 1 views) whose points chain
    through view_offsets (and whose super-block sums use both parity
    buffers).  Views on both sides of the group boundary bit-exact vs the
    oracle."""
    from structured_light_for_3d_model_replication_amd import synth
    V, H, W = 33, 1080, 1920
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    stacks, texes = [], []
    for v in range(V):
        s, t = synth.render_stack(rig, seed=300 + v, view_deg=11.0 * v, device="cuda")
        stacks.append(s)
        texes.append(t)
    eng.set_calibration(cal, H, W)
    res = eng.decode_triangulate(torch.stack(stacks), texture=torch.stack(texes), maps=False, cloud=True,
                                 xyz_dtype=torch.float32)
    eng.sync()
    assert eng.last_launch_info()[1] == 2
    xyz, bgr, off = _cloud_np(res["cloud"])
    for v in (0, 31, 32):  # first view, last view of group 0, the view of group 1
        sth, texh = stacks[v].cpu().numpy(), texes[v].cpu().numpy()
        _, _, _, P, C = o.decode_triangulate(list(sth), texh, cal)
        assert off[v + 1] - off[v] == len(P)
        _assert_f32(xyz[off[v]:off[v + 1]], P)
        np.testing.assert_array_equal(bgr[off[v]:off[v + 1]], C)
    assert np.all(np.diff(off) > 0)


def test_huge_view_plane_descriptors(eng):
    """A 8000x6000 view with 11 + 11 bits: its 46 planes span 2.2 GB (> 2 GiB),
    so k_decode reads them through a descriptor per plane.  The fixed-mask
    maps of sampled rows equal the oracle's decode of those rows (a per-pixel
    computation), and the cloud's point count equals the decided mask's."""
    from structured_light_for_3d_model_replication_amd import synth
    H, W = 6000, 8000
    rig = synth.Rig(H=H, W=W)
    st, tex = synth.render_stack(rig, seed=77, device="cuda")
    assert st.shape[0] * H * W >= 2 ** 31
    cal = synth.make_calibration(rig)
    eng.set_calibration(cal, H, W)
    res = eng.decode_triangulate(st, texture=tex, mask_mode="fixed", maps=True, cloud=True,
                                 xyz_dtype=torch.float32, fast_f32=True)
    eng.sync()
    rows = [0, 1, 2999, 4321, 5999]
    sub = st[:, rows, :].cpu().numpy()
    col, row, mask = o.gray_decode_images(list(sub), 1920, 1080, o.MASK_FIXED)
    np.testing.assert_array_equal(res["col_map"][0][rows].cpu().numpy(), col)
    np.testing.assert_array_equal(res["row_map"][0][rows].cpu().numpy(), row)
    np.testing.assert_array_equal(res["mask"][0][rows].cpu().numpy(), mask)
    n = res["cloud"].total()
    assert 0 < n <= int(res["mask"][0].sum())


def test_wide_projector_13bit(eng):
    """A 5000-column projector
    (13-bit codes, 15-bit records, the generic decode kernel)."""
    rig, st, tex, cal = _render(160, 256, 5000, 1080, seed=17)
    sth, texh = st.cpu().numpy(), tex.cpu().numpy()
    col, row, mask, P, C = o.decode_triangulate(list(sth), texh, cal, 5000, 1080)
    res = _run(eng, sth, texh, cal, 5000, 1080, xyz_dtype=torch.float64)
    np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
    np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask)
    xyz, bgr, off = _cloud_np(res["cloud"])
    assert off[-1] == len(P)
    np.testing.assert_array_equal(xyz.view(np.uint64), P.view(np.uint64))
    np.testing.assert_array_equal(bgr, C)


def test_three_launch_groups_maps_and_cloud(eng):
    """Three launch groups in one call (20 views of 1920x1080 at 16K chunks per
    group: 8 + 8 + 4 views), the histogram parity buffers alternating across
    groups and across two back-to-back calls: every view's maps (adaptive
    thresholds) and cloud bit-exact vs the oracle, view_offsets chained over
    all groups."""
    from structured_light_for_3d_model_replication_amd import synth
    V, H, W = 20, 1080, 1920
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    stacks, texes = [], []
    for v in range(V):
        s, t = synth.render_stack(rig, seed=500 + v, view_deg=18.0 * v, device="cuda")
        stacks.append(s)
        texes.append(t)
    st, tx = torch.stack(stacks), torch.stack(texes)
    eng.set_calibration(cal, H, W)
    out = {}
    for call in range(2):
        res = eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32, out=out)
        eng.sync()
        xyz, bgr, off = _cloud_np(res["cloud"])
        assert off[0] == 0 and np.all(np.diff(off) > 0)
        views = range(V) if call == 0 else (0, 8, 16, 19)
        for v in views:
            sth, texh = stacks[v].cpu().numpy(), texes[v].cpu().numpy()
            col, row, mask, P, C = o.decode_triangulate(list(sth), texh, cal)
            np.testing.assert_array_equal(res["col_map"][v].cpu().numpy(), col)
            np.testing.assert_array_equal(res["row_map"][v].cpu().numpy(), row)
            np.testing.assert_array_equal(res["mask"][v].cpu().numpy(), mask)
            assert off[v + 1] - off[v] == len(P), f"view {v}"
            _assert_f32(xyz[off[v]:off[v + 1]], P)
            np.testing.assert_array_equal(bgr[off[v]:off[v + 1]], C)


def test_multigroup_call_on_a_caller_stream(eng):
    """A multi-group call on a non-default caller stream: work queued behind
    it on that stream sees the finished cloud (single-stream semantics)."""
    from structured_light_for_3d_model_replication_amd import synth
    V, H, W = 18, 1080, 1920
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    st = torch.stack([synth.render_stack(rig, seed=700 + v, view_deg=20.0 * v, device="cuda")[0]
                      for v in range(V)])
    eng.set_calibration(cal, H, W)
    ref = eng.decode_triangulate(st, maps=False, cloud=True, xyz_dtype=torch.float32)
    eng.sync()
    ref_off = ref["cloud"].offsets().copy()
    ref_sum = float(ref["cloud"].xyz[: ref_off[-1]].double().sum())
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        res = eng.decode_triangulate(st, maps=False, cloud=True, xyz_dtype=torch.float32, stream=s)
        n = res["cloud"].view_offsets[-1].clone()  # queued on s behind the call
        tot = res["cloud"].xyz[: int(ref_off[-1])].double().sum()
    s.synchronize()
    assert int(n.item()) == ref_off[-1]
    assert float(tot.item()) == ref_sum


def test_time_kernels_keeps_outputs_and_later_calls_exact(eng):
    """sl_time_kernels (measurement) re-runs the last call's kernels: positive
    durations, the call's outputs unchanged, and the next call (histograms
    reset) still bit-exact."""
    rig, st, tex, cal = _render(480, 640, 1920, 1080, seed=21)
    sth, texh = st.cpu().numpy(), tex.cpu().numpy()
    col, row, mask, P, C = o.decode_triangulate(list(sth), texh, cal)
    for _ in range(2):
        res = _run(eng, sth, texh, cal, 1920, 1080, xyz_dtype=torch.float32)
        t = eng.time_kernels(3)
        assert all(x > 0 for x in t)
        eng.sync()
        np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
        np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask)
        xyz, bgr, off = _cloud_np(res["cloud"])
        assert off[-1] == len(P)
        _assert_f32(xyz, P)
        np.testing.assert_array_equal(bgr, C)
    with pytest.raises(ValueError):
        eng.time_kernels(3)  # nothing left to re-run


@pytest.mark.parametrize("shift", [0, 16, 48])
def test_colour_quads_caller_buffers(eng, shift):
    """k_cloud's colour quads (4 consecutive points per lane, one dwordx3) take
    the quad phase from the chunk's first colour byte address, 3 x its first
    point's index (every phase mod 4 occurs across a frame's chunks), with the
    points before the first quad and after the last stored byte by byte: two
    views, maps + cloud and cloud only, caller buffers at several 16-byte
    aligned offsets -- colours, xyz and offsets equal to the oracle's
    (sl_system.py:651, C = texture[idx]), no byte outside the cloud written.
    A buffer that is not 16-byte aligned is refused (sl_decode_triangulate)."""
    rig, st0, tex0, cal = _render(96, 256, 1920, 1080, seed=41)
    _, st1, tex1, _ = _render(96, 256, 1920, 1080, seed=42, view=10.0)
    st = torch.stack([st0, st1])
    tx = torch.stack([tex0, tex1])
    eng.set_calibration(cal, 96, 256)
    cap = 2 * 96 * 256
    for maps in (True, False):
        big = torch.full((3 * cap + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        bgr = big[shift:shift + 3 * cap].view(cap, 3)
        out = {"xyz": torch.empty((cap, 3), dtype=torch.float32, device="cuda"), "bgr": bgr,
               "view_offsets": torch.empty(3, dtype=torch.int64, device="cuda")}
        res = eng.decode_triangulate(st, 1920, 1080, texture=tx, maps=maps, cloud=True, out=out)
        eng.sync()
        assert res["cloud"].bgr.data_ptr() == big.data_ptr() + shift
        xyz, col, off = _cloud_np(res["cloud"])
        for v, (s_, t_) in enumerate(((st0, tex0), (st1, tex1))):
            _, _, _, P, C = o.decode_triangulate(list(s_.cpu().numpy()), t_.cpu().numpy(), cal)
            assert off[v + 1] - off[v] == len(P)
            np.testing.assert_array_equal(col[off[v]:off[v + 1]], C)
            _assert_f32(xyz[off[v]:off[v + 1]], P)
        tail = big[shift + 3 * int(off[-1]):].cpu().numpy()
        assert np.all(tail == 0xA5), "bytes past the cloud were written"
        if shift:
            assert np.all(big[:shift].cpu().numpy() == 0xA5), "bytes before the buffer were written"
    assert len(P) > 1000  # 48 chunks over both views: many quads, heads and tails
    big = torch.empty((3 * cap + 8,), dtype=torch.uint8, device="cuda")
    bad = {"xyz": torch.empty((cap, 3), dtype=torch.float32, device="cuda"),
           "bgr": big[1:1 + 3 * cap].view(cap, 3), "view_offsets": torch.empty(3, dtype=torch.int64, device="cuda")}
    with pytest.raises(ValueError):
        eng.decode_triangulate(st, 1920, 1080, texture=tx, maps=False, cloud=True, out=bad)


def test_full_12mp_posed_views_cloud_only_vs_oracle(eng):
    """Config 4/5 shapes at full size: two 4000x3000 views (12 MP, 11+11 bits,
    cloud only: the row planes are never read) with the turntable pose
    epilogue, in one call (one launch group per view); f64 xyz bit-identical
    to the oracle, merged order and per-view offsets."""
    from structured_light_for_3d_model_replication_amd import synth
    V, H, W = 2, 3000, 4000
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig, with_Nc=False)
    stacks, texes = [], []
    for v in range(V):
        s, t = synth.render_stack(rig, seed=900 + v, view_deg=1.0 * v, device="cuda")
        stacks.append(s)
        texes.append(t)
    poses = np.stack([synth.turntable_pose(1.0 * v) for v in range(V)])
    eng.set_calibration(cal, H, W)
    res = eng.decode_triangulate(torch.stack(stacks), texture=torch.stack(texes), maps=False, cloud=True,
                                 xyz_dtype=torch.float64, poses=torch.from_numpy(poses).cuda())
    eng.sync()
    xyz, bgr, off = _cloud_np(res["cloud"])
    assert off[0] == 0
    for v in range(V):
        _, _, _, P, C = o.decode_triangulate(list(stacks[v].cpu().numpy()), texes[v].cpu().numpy(), cal,
                                             pose=poses[v])
        assert off[v + 1] - off[v] == len(P)
        np.testing.assert_array_equal(xyz[off[v]:off[v + 1]].view(np.uint64), P.view(np.uint64))
        np.testing.assert_array_equal(bgr[off[v]:off[v + 1]], C)


@pytest.mark.parametrize("H,W", [(1, 1), (1, 17), (3, 1), (2, 1023), (1, 1025), (5, 64)])
def test_tiny_and_ragged_frames_vs_oracle(eng, H, W):
    """Degenerate frame shapes: single pixel, single row / column, a chunk
    boundary straddled by one pixel (1023, 1025 px); maps and cloud bit-exact
    vs the oracle (adaptive thresholds over so few pixels included)."""
    rig, st, tex, cal = _render(H, W, 1920, 1080, seed=H * 1000 + W, device="cpu")
    sth, texh = st.numpy(), tex.numpy()
    col, row, mask, P, C = o.decode_triangulate(list(sth), texh, cal)
    res = _run(eng, sth, texh, cal, 1920, 1080, xyz_dtype=torch.float64)
    np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
    np.testing.assert_array_equal(res["row_map"][0].cpu().numpy(), row)
    np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask)
    xyz, bgr, off = _cloud_np(res["cloud"])
    assert off[-1] == len(P)
    np.testing.assert_array_equal(xyz.view(np.uint64), P.view(np.uint64))
    np.testing.assert_array_equal(bgr, C)


def test_views_ending_inside_a_chunk_every_view_vs_oracle(eng):
    """A three-view batch whose views end inside a chunk (HW % 1024 != 0, the
    16-byte path), maps + cloud (strided decode grid, pixel-order records) and
    cloud only (dynamic grid, chunk-slot records), f64 and f32-fast xyz: every
    view's maps, mask, thresholds and points equal to the oracle's, and the
    two paths' clouds equal to each other."""
    from structured_light_for_3d_model_replication_amd import synth
    H, W = 517, 1200  # HW % 16 == 0 (16-byte path), HW % 1024 != 0
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig, with_Nc=False)
    sts, txs = zip(*[synth.render_stack(rig, seed=970 + v, view_deg=15.0 * v, device="cuda") for v in range(3)])
    st, tx = torch.stack(sts), torch.stack(txs)
    eng.set_calibration(cal, H, W)
    refs = [o.decode_triangulate(list(sts[v].cpu().numpy()), txs[v].cpu().numpy(), cal) for v in range(3)]
    clouds = {}
    for maps in (True, False):
        for fast in (False, True):
            kw = dict(fast_f32=True) if fast else dict(xyz_dtype=torch.float64)
            r = eng.decode_triangulate(st, texture=tx, maps=maps, cloud=True, **kw)
            eng.sync()
            xyz, bgr, off = _cloud_np(r["cloud"])
            clouds[(maps, fast)] = (xyz, bgr, off)
            for v in range(3):
                col, row, mask, P, C = refs[v]
                assert off[v + 1] - off[v] == len(P)
                if fast:
                    _assert_fast(xyz[off[v]:off[v + 1]], P)
                else:
                    np.testing.assert_array_equal(xyz[off[v]:off[v + 1]].view(np.uint64), P.view(np.uint64))
                np.testing.assert_array_equal(bgr[off[v]:off[v + 1]], C)
                if maps:
                    np.testing.assert_array_equal(r["col_map"][v].cpu().numpy(), col)
                    np.testing.assert_array_equal(r["row_map"][v].cpu().numpy(), row)
                    np.testing.assert_array_equal(r["mask"][v].cpu().numpy(), mask)
    for fast in (False, True):
        for a_, b_ in zip(clouds[(True, fast)], clouds[(False, fast)]):
            np.testing.assert_array_equal(a_, b_)


@pytest.mark.parametrize("val", ["1", "2", "4", "64", "255"])
def test_debug_env_cannot_change_results(monkeypatch, val):
    """No environment variable selects a kernel variant (the rejected
    variants are gone from the library; only SLGPU_VERIFY32, a test switch,
    is read): a context created with SLGPU_DEBUG set still gives oracle-exact
    maps and cloud."""
    from structured_light_for_3d_model_replication_amd import core
    monkeypatch.setenv("SLGPU_DEBUG", val)
    e = core.Reconstructor(torch.device("cuda", 0))
    try:
        rig, st, tex, cal = _render(96, 128, 1920, 1080, seed=31)
        sth, texh = st.cpu().numpy(), tex.cpu().numpy()
        col, row, mask, P, C = o.decode_triangulate(list(sth), texh, cal)
        for dt in (torch.float64, torch.float32):
            res = _run(e, sth, texh, cal, 1920, 1080, xyz_dtype=dt)
            np.testing.assert_array_equal(res["col_map"][0].cpu().numpy(), col)
            np.testing.assert_array_equal(res["mask"][0].cpu().numpy(), mask)
            xyz, bgr, off = _cloud_np(res["cloud"])
            assert off[-1] == len(P)
            if dt == torch.float64:
                np.testing.assert_array_equal(xyz.view(np.uint64), P.view(np.uint64))
            else:
                _assert_f32(xyz, P)
            np.testing.assert_array_equal(bgr, C)
    finally:
        e.close()


def test_calibration_cache_sees_every_nc_column(eng):
    """Two non-pinhole Nc tables that differ only in columns a sampled key
    would skip, and an Nc mutated in place between calls: each call uses the
    table it was given (oracle-exact f64 clouds)."""
    rig, st, tex, cal = _render(120, 160, 1920, 1080, seed=78)
    sth, texh = st.cpu().numpy(), tex.cpu().numpy()
    rng = np.random.default_rng(1)
    base = dict(cal)
    base["Nc"] = cal["Nc"] * (1.0 + 1e-3 * rng.standard_normal(cal["Nc"].shape))
    other = dict(base)
    other["Nc"] = base["Nc"].copy()
    _, _, mask, _, _ = o.decode_triangulate(list(sth), texh, base)
    idx = np.flatnonzero(mask.ravel())
    cols = idx[(idx % 7) == 3][:50]          # valid pixels, not on any sampling stride
    other["Nc"][:, cols] *= 1.01
    for cal_i in (base, other, base):
        _, _, _, P, C = o.decode_triangulate(list(sth), texh, cal_i)
        res = _run(eng, sth, texh, cal_i, 1920, 1080)
        xyz, bgr, off = _cloud_np(res["cloud"])
        assert off[-1] == len(P)
        np.testing.assert_array_equal(xyz.view(np.uint64), P.view(np.uint64))
    # in place: same dict, same array object, new contents
    base["Nc"][:, cols] *= 0.99
    _, _, _, P, C = o.decode_triangulate(list(sth), texh, base)
    res = _run(eng, sth, texh, base, 1920, 1080)
    xyz, _, off = _cloud_np(res["cloud"])
    assert off[-1] == len(P)
    np.testing.assert_array_equal(xyz.view(np.uint64), P.view(np.uint64))


@pytest.mark.parametrize("H,W,mode,maps,cloud", [
    (240, 320, "adaptive", False, True),   # decide path, cloud only
    (240, 320, "fixed", True, True),       # decide path, maps + cloud
    (240, 320, "adaptive", True, False),   # decide path, maps only
    (250, 333, "adaptive", False, True),   # byte path: k_decode + k_count + k_cloud
    (250, 333, "fixed", True, False),
])
def test_mask_counts_match_the_oracle(eng, H, W, mode, maps, cloud):
    """sl_mask_counts_to: the per-view count of masked-in pixels (the N of
    "Processing N valid pixels...", sl_system.py:601-602) over a 3-view batch,
    on every kernel path; a later call without it counts nothing."""
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    sts = [synth.render_stack(rig, seed=60 + v, view_deg=5.0 * v)[0] for v in range(3)]
    want = [int(o.gray_decode_images(list(s.numpy()), 1920, 1080, mode)[2].sum()) for s in sts]
    eng.set_calibration(cal, H, W)
    st = torch.stack(sts).cuda()
    mc = torch.full((3,), -7, dtype=torch.int64, device="cuda")
    eng.decode_triangulate(st, 1920, 1080, mask_mode=mode, maps=maps, cloud=cloud, mask_counts=mc)
    eng.sync()
    assert mc.cpu().tolist() == want
    mc.fill_(-7)
    eng.decode_triangulate(st, 1920, 1080, mask_mode=mode, maps=maps, cloud=cloud)
    eng.sync()
    assert mc.cpu().tolist() == [-7, -7, -7]


@pytest.mark.parametrize("f_scale", [0.9, 0.2])
def test_verified_f32_route_equals_the_exact_sequence(f_scale, monkeypatch):
    """SL_XYZ_F32 through the verified shorter f64 route (M_VERIFY: P' =
    (x, y, 1) * -w / (n . (x, y, 1)), no ray normalisation, the float32
    rounding proven unambiguous, else the operators' sequences) == the exact
    sequence (SLGPU_VERIFY32=0) == float32 of the oracle's f64, on a 1080p
    view; f_scale 0.2 is a wide-angle camera (|x| up to 2.5)."""
    from structured_light_for_3d_model_replication_amd import core, synth
    rig, st, tex, cal = _render(1080, 1920, 1920, 1080, seed=404)
    cal = dict(cal)
    K = np.array(cal["cam_K"], dtype=np.float64)
    K[0, 0] = K[1, 1] = f_scale * rig.W
    cal["cam_K"] = K
    cal["Nc"] = np.zeros((3, 1))  # no per-pixel table: rays from cam_K (sl_system.py:607-621)
    sth, texh = st.cpu().numpy(), tex.cpu().numpy()
    _, _, _, P, C = o.decode_triangulate(list(sth), texh, cal, 1920, 1080)
    outs = []
    for verify in ("1", "0"):
        monkeypatch.setenv("SLGPU_VERIFY32", verify)
        e = core.Reconstructor(torch.device("cuda", 0))
        try:
            res = _run(e, sth, texh, cal, 1920, 1080, xyz_dtype=torch.float32, maps=False)
            xyz, bgr, off = _cloud_np(res["cloud"])
            assert off[-1] == len(P) > 100_000
            _assert_f32(xyz, P)
            np.testing.assert_array_equal(bgr, C)
            outs.append(xyz)
        finally:
            e.close()
    np.testing.assert_array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


def _snap(res):
    """Host copies of a call's maps and cloud (after a sync)."""
    xyz, bgr, off = _cloud_np(res["cloud"])
    return (res["col_map"].cpu().numpy(), res["row_map"].cpu().numpy(), res["mask"].cpu().numpy(), xyz, bgr, off)


def test_stack_ready_calls_bit_identical():
    """sl_stack_ready: back-to-back calls over different views on one context,
    each declaring its stack ready (resident, or ready once an event recorded
    after a copy on another stream completes: the call waits for it on its
    stream), interleaved with a plain call and a fixed-mask call, nothing
    synchronised in between: every call's maps, mask thresholds and cloud
    bit-identical to the same call made alone, and view 0's to the oracle."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W = 480, 640
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    views = [synth.render_stack(rig, seed=900 + v, view_deg=25.0 * v, device="cuda") for v in range(5)]
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    modes = ["adaptive", "adaptive", "fixed", "adaptive", "adaptive"]
    ref = []
    for (st, tx), mm in zip(views, modes):
        ref.append(_snap(eng.decode_triangulate(st, texture=tx, mask_mode=mm, maps=True, cloud=True,
                                                xyz_dtype=torch.float32, out={})))
        eng.sync()
    side = torch.cuda.Stream()
    for rep in range(2):
        outs, res, keep = [{} for _ in views], [], []
        for i, ((st, tx), mm) in enumerate(zip(views, modes)):
            ready = True if i != 2 or rep == 1 else None
            if i == 3:  # the stack arrives by a copy on another stream; the event marks it ready
                buf = torch.empty_like(st)
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    buf.copy_(st)
                    ev = torch.cuda.Event()
                    ev.record(side)
                # (the call's stream does not wait for the copy: the call waits
                # for the event, sl_stack_ready)
                keep.append(buf)
                st, ready = buf, ev
            res.append(eng.decode_triangulate(st, texture=tx, mask_mode=mm, maps=True, cloud=True,
                                              xyz_dtype=torch.float32, out=outs[i], stack_ready=ready))
        eng.sync()
        for i, r in enumerate(res):
            got = _snap(r)
            for a, b in zip(got, ref[i]):
                np.testing.assert_array_equal(a, b, err_msg=f"call {i}, rep {rep}")
    st, tx = views[0]
    col, row, mask, P, C = o.decode_triangulate(list(st.cpu().numpy()), tx.cpu().numpy(), cal)
    np.testing.assert_array_equal(ref[0][0][0], col)
    np.testing.assert_array_equal(ref[0][2][0], mask)
    _assert_f32(ref[0][3], P)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_verified_route_random_planes_and_poses(seed, monkeypatch):
    """The verified f32 route on adversarial inputs through
    triangulate_maps: a random camera (centre off the grid), a random plane
    table (random normals, |w| from 1e-3 to 1e6, some planes nearly parallel
    to the rays: large kappa), random column codes on every pixel, with and
    without a random pose whose translation cancels most of the point (the
    posed interval test's fallback) -- float32 output bit-identical to the
    exact sequence (SLGPU_VERIFY32=0) and to float32 of the oracle's f64."""
    from structured_light_for_3d_model_replication_amd import core
    rng = np.random.default_rng(seed)
    H, W, Wp = 64, 256, 512
    # centres half a pixel off the grid (|x|, |y| >= 2^-20: the route's range premise holds)
    cx, cy = rng.integers(0, W) + 0.5 + rng.uniform(-0.1, 0.1), rng.integers(0, H) + 0.5 + rng.uniform(-0.1, 0.1)
    K = np.array([[rng.uniform(100, 2000), 0, cx], [0, rng.uniform(100, 2000), cy], [0, 0, 1]], dtype=np.float64)
    n = rng.normal(size=(Wp, 3))
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    n[: Wp // 8, 2] *= 1e-3  # nearly parallel to the optical axis' planes
    w = rng.choice([-1.0, 1.0], size=Wp) * 10.0 ** rng.uniform(-3, 6, size=Wp)
    planes = np.concatenate([n, w[:, None]], axis=1)
    cal = {"Nc": np.zeros((3, 1)), "Oc": np.zeros((3, 1)), "wPlaneCol": planes.T.copy(), "cam_K": K}
    col = rng.integers(0, Wp, size=(H, W), dtype=np.int32)
    mask = np.ones((H, W), dtype=bool)
    tex = rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    P, C = o.reconstruct_point_cloud(col, np.zeros_like(col), mask, tex, cal)
    c = P.mean(axis=0)
    R = np.linalg.qr(rng.normal(size=(3, 3)))[0]
    pose = np.eye(4)
    pose[:3, :3] = R
    pose[:3, 3] = -(R @ c) + rng.normal(size=3) * 1e-3  # most points land near the origin
    outs = {}
    for verify in ("1", "0"):
        monkeypatch.setenv("SLGPU_VERIFY32", verify)
        e = core.Reconstructor(torch.device("cuda", 0))
        try:
            e.set_calibration(cal, H, W)
            for posed in (False, True):
                cl = e.triangulate_maps(torch.from_numpy(col), torch.from_numpy(mask), torch.from_numpy(tex),
                                        xyz_dtype=torch.float32,
                                        poses=torch.from_numpy(pose[None]) if posed else None)
                e.sync()
                outs[(verify, posed)] = _cloud_np(cl)
        finally:
            e.close()
    for posed in (False, True):
        a, b = outs[("1", posed)], outs[("0", posed)]
        np.testing.assert_array_equal(a[2], b[2])
        np.testing.assert_array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
        want = o.apply_pose(P, pose) if posed else P
        assert a[2][-1] == len(want)
        np.testing.assert_array_equal(a[0], want.astype(np.float32))
        np.testing.assert_array_equal(a[1], C)
