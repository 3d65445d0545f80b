"""sl_stack_next (pre-stats): a call's k_cloud also runs the NEXT call's
adaptive-mask histogram pass (sl_system.py:526-528), so that call starts with
its decode.  Bar: every call's maps, mask, thresholds and cloud bit-identical
to the same call made alone, whatever the chain does (declared stacks taken,
mismatched declarations ignored, fixed-mask calls in between, multi-group
calls, the pool's prepared calls, kernel re-runs in between), and the oracle's
on a sample (GPU only)."""
import numpy as np
import pytest
import torch

from oracle import sl_oracle as o

pytestmark = pytest.mark.gpu


def _snap(res, eng):
    cloud = res["cloud"]
    off = cloud.offsets()
    out = [cloud.xyz[: off[-1]].cpu().numpy(), cloud.bgr[: off[-1]].cpu().numpy(), np.asarray(off)]
    if "col_map" in res:
        out += [res["col_map"].cpu().numpy(), res["row_map"].cpu().numpy(), res["mask"].cpu().numpy()]
    out.append(np.array(eng.last_thresholds(0), dtype=np.float64))
    return out


def _same(got, ref, what):
    for k, (a, b) in enumerate(zip(got, ref)):
        np.testing.assert_array_equal(a, b, err_msg=f"{what}: output {k}")


def test_chained_calls_bit_identical():
    """Five views, each call naming the next one's stack: adaptive calls take
    the histograms computed by the previous call's k_cloud; a declaration that
    does not match the next call (another buffer) is ignored; a fixed-mask call
    in the chain consumes nothing but still queues the pass for its successor;
    three rounds of it."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W = 480, 640
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    views = [synth.render_stack(rig, seed=700 + v, view_deg=20.0 * v, device="cuda") for v in range(5)]
    modes = ["adaptive", "adaptive", "fixed", "adaptive", "adaptive"]
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    ref = []
    for (st, tx), mm in zip(views, modes):
        r = eng.decode_triangulate(st, texture=tx, mask_mode=mm, maps=True, cloud=True, xyz_dtype=torch.float32,
                                   out={})
        eng.sync()
        ref.append(_snap(r, eng))
    decoy = views[0][0].clone()  # same content, another buffer: the declaration must not be taken for it
    for rnd in range(3):
        for i, ((st, tx), mm) in enumerate(zip(views, modes)):
            nxt = views[(i + 1) % len(views)][0]
            if rnd == 1 and i == 1:
                nxt = decoy  # call 2 is on views[2]: computes its own (fixed mask anyway)
            if rnd == 1 and i == 2:
                nxt = decoy  # call 3 is on views[3], not the decoy: k_stats runs
            r = eng.decode_triangulate(st, texture=tx, mask_mode=mm, maps=True, cloud=True,
                                       xyz_dtype=torch.float32, out={}, next_stack=nxt)
            eng.sync()
            _same(_snap(r, eng), ref[i], f"round {rnd}, call {i}")
    st, tx = views[1]
    col, row, mask, P, C = o.decode_triangulate(list(st.cpu().numpy()), tx.cpu().numpy(), cal)
    np.testing.assert_array_equal(ref[1][3][0], col)
    np.testing.assert_array_equal(ref[1][5][0], mask)
    np.testing.assert_array_equal(ref[1][0], P.astype(np.float32))


def test_chained_calls_without_syncs():
    """The same chain queued back to back (no host sync between calls, each
    call into its own outputs): the pass a call's k_cloud runs and the next
    call's decode are ordered by the stream alone."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W = 240, 320
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    views = [synth.render_stack(rig, seed=40 + v, view_deg=33.0 * v, device="cuda") for v in range(4)]
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    ref = []
    for st, tx in views:
        r = eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32, out={})
        eng.sync()
        ref.append(_snap(r, eng))
    order = [0, 1, 2, 3, 3, 2, 1, 0, 0, 1]
    res = []
    for k, v in enumerate(order):
        st, tx = views[v]
        nxt = views[order[k + 1]][0] if k + 1 < len(order) else None
        res.append(eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32, out={},
                                          next_stack=nxt))
    eng.sync()
    for k, (v, r) in enumerate(zip(order, res)):
        _same(_snap(r, eng)[:-1], ref[v][:-1], f"call {k} (view {v})")


def test_chained_multi_group_calls():
    """Calls of two launch groups (34 1080p views: 32 + 2): the last group's
    k_cloud computes the histograms of the next call's first group (32 views);
    within each call the first group's k_cloud computes the second group's."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W, V = 1080, 1920, 34
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig, with_Nc=False)
    base = [synth.render_stack(rig, seed=60 + v, view_deg=40.0 * v, device="cuda", include_rows=False)
            for v in range(3)]
    n_img = base[0][0].shape[0]
    A = torch.empty((V, n_img, H, W), dtype=torch.uint8, device="cuda")
    TA = torch.empty((V, H, W, 3), dtype=torch.uint8, device="cuda")
    for v in range(V):
        A[v].copy_(base[v % 3][0])
        TA[v].copy_(base[v % 3][1])
    B, TB = A.roll(1, 0).contiguous(), TA.roll(1, 0).contiguous()
    del base
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    ref = {}
    for name, (st, tx) in {"A": (A, TA), "B": (B, TB)}.items():
        r = eng.decode_triangulate(st, texture=tx, cloud=True, xyz_dtype=torch.float32, out={})
        eng.sync()
        assert eng.last_launch_info()[1] == 2
        ref[name] = _snap(r, eng)
    for k, (name, (st, tx), nxt) in enumerate([("A", (A, TA), B), ("B", (B, TB), A), ("A", (A, TA), None)]):
        r = eng.decode_triangulate(st, texture=tx, cloud=True, xyz_dtype=torch.float32, out={}, next_stack=nxt)
        eng.sync()
        _same(_snap(r, eng)[:-1], ref[name][:-1], f"call {k} ({name})")


def test_chain_survives_kernel_reruns():
    """sl_time_kernels between chained calls (it rebuilds the inputs the call
    consumed, re-runs the last group's kernels without the pre-stats
    workgroups and drops the queued pass): the next call computes its own
    histograms, bit-identical results."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W = 480, 640
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    st, tx = synth.render_stack(rig, seed=5, view_deg=10.0, device="cuda")
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    r = eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32, out={})
    eng.sync()
    ref = _snap(r, eng)
    for k in range(3):
        r = eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32, out={},
                                   next_stack=st)
        eng.sync()
        _same(_snap(r, eng), ref, f"call {k}")
        eng.time_kernels(3)


def test_pool_prepared_calls_with_next_stack():
    """ReconstructorPool's resident-input path (prepared calls per lane), each
    call naming the stack of its lane's next call, the bench's c3 / c4 / c5
    shape: every call's cloud equal to the plain engine's."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W, V = 240, 320, 3
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    sts = [synth.render_stack(rig, seed=80 + v, view_deg=15.0 * v, device="cuda") for v in range(V)]
    stack = torch.stack([s for s, _ in sts])
    tex = torch.stack([t for _, t in sts])
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    r = eng.decode_triangulate(stack, texture=tex, maps=True, cloud=True, xyz_dtype=torch.float32, out={})
    eng.sync()
    ref = _snap(r, eng)[:-1]
    pool = core.ReconstructorPool(torch.device("cuda", 0), lanes=2, reuse_outputs=True)
    pool.set_calibration(cal, H, W)
    for k in range(6):
        res = pool.decode_triangulate(stack, texture=tex, maps=True, cloud=True, xyz_dtype=torch.float32,
                                      wait_inputs=False, next_stack=stack)
        pool.sync()
        _same(_snap(res, pool.engines[res["lane"]])[:-1], ref, f"pool call {k}")


def test_next_stack_argument_checks():
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W = 96, 128
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    st, tx = synth.render_stack(rig, seed=1, device="cuda")
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    with pytest.raises(ValueError):
        eng.decode_triangulate(st, texture=tx, next_stack=st[:, :, : W // 2])  # another frame size
    with pytest.raises(ValueError):
        eng.decode_triangulate(st, texture=tx, next_stack=st.float())
    with pytest.raises(Exception):  # 16-byte alignment (sl_stack_next)
        flat = torch.empty(st.numel() + 1, dtype=torch.uint8, device="cuda")
        eng.decode_triangulate(st, texture=tx, next_stack=flat[1:].view(st.shape))


def test_graph_captured_chain():
    """bench.py's headline window: K chained calls (next_stack) captured into
    a hipGraph on a side stream after eager calls on it, replayed once, then
    eager calls again -- every call's outputs equal to the plain call's; and
    a dropped chain (drop_next) computes its own histograms."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W = 480, 640
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    st, tx = synth.render_stack(rig, seed=11, view_deg=5.0, device="cuda")
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    ref = _snap(eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32, out={}),
                eng)
    s = torch.cuda.Stream()
    outs = [{} for _ in range(5)]
    with torch.cuda.stream(s):
        for o in outs:  # eager calls (allocate the outputs), chained
            eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32, out=o,
                                   next_stack=st)
    torch.cuda.synchronize()
    for o in outs:
        for v in o.values():
            v.zero_()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    res = []
    with torch.cuda.graph(g, stream=s):
        for o in outs:
            res.append(eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32,
                                              out=o, next_stack=st))
    with torch.cuda.stream(s):
        g.replay()
    torch.cuda.synchronize()
    for k, r in enumerate(res):
        _same(_snap(r, eng)[:-1], ref[:-1], f"graph call {k}")
    with torch.cuda.stream(s):  # eager again after the replay, then a dropped chain
        r = eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32, out={},
                                   next_stack=st)
        eng.drop_next()
        r2 = eng.decode_triangulate(st, texture=tx, maps=True, cloud=True, xyz_dtype=torch.float32, out={})
    torch.cuda.synchronize()
    _same(_snap(r, eng)[:-1], ref[:-1], "eager after replay")
    _same(_snap(r2, eng)[:-1], ref[:-1], "after drop_next")


def _group_views(H, W, V, maps, seed0):
    """V resident views cycling through 3 rendered ones (stack, texture), the
    3 base views, and their single-view clouds/maps (one launch group each)."""
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.Rig(H=H, W=W)
    base = [synth.render_stack(rig, seed=seed0 + v, view_deg=50.0 * v, device="cuda", include_rows=maps)
            for v in range(3)]
    n_img = base[0][0].shape[0]
    A = torch.empty((V, n_img, H, W), dtype=torch.uint8, device="cuda")
    TA = torch.empty((V, H, W, 3), dtype=torch.uint8, device="cuda")
    for v in range(V):
        A[v].copy_(base[v % 3][0])
        TA[v].copy_(base[v % 3][1])
    return rig, base, A, TA


@pytest.mark.parametrize("maps", [False, True])
def test_multi_group_call_prestats_between_groups(maps):
    """One call of three launch groups (70 1080p views: 32 + 32 + 6): groups 2
    and 3 take the histograms the previous group's k_cloud computed (no k_stats
    launch).  Every view's thresholds, cloud slice (and maps) equal those of
    the same view decoded alone; one view of the last group against the
    oracle."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W, V = 1080, 1920, 70
    rig, base, A, TA = _group_views(H, W, V, maps, 300)
    cal = synth.make_calibration(rig, with_Nc=False)
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    single = []
    for st, tx in base:
        r = eng.decode_triangulate(st, texture=tx, maps=maps, cloud=True, xyz_dtype=torch.float32, out={})
        eng.sync()
        single.append(_snap(r, eng))
    kw = dict(texture=TA, maps=maps, cloud=True, xyz_dtype=torch.float32)
    r = eng.decode_triangulate(A, out={}, **kw)
    eng.sync()
    assert eng.last_launch_info()[1] == 3
    got = _snap(r, eng)[:-1]
    off = got[2]
    for v in range(V):
        ref = single[v % 3]
        n = ref[2][1]
        np.testing.assert_array_equal(got[0][off[v]:off[v + 1]], ref[0][:n], err_msg=f"view {v} xyz")
        np.testing.assert_array_equal(got[1][off[v]:off[v + 1]], ref[1][:n], err_msg=f"view {v} bgr")
        if maps:
            for k in (3, 4, 5):
                np.testing.assert_array_equal(got[k][v], ref[k][0], err_msg=f"view {v} map {k}")
        np.testing.assert_array_equal(np.array(eng.last_thresholds(v), dtype=np.float64), ref[-1],
                                      err_msg=f"view {v} thresholds")
    v = 67  # last group
    col, row, mask, P, C = o.decode_triangulate(list(A[v].cpu().numpy()), TA[v].cpu().numpy(), cal)
    np.testing.assert_array_equal(got[0][off[v]:off[v + 1]], P.astype(np.float32))
    np.testing.assert_array_equal(got[1][off[v]:off[v + 1]], C)


def test_failed_call_consumes_queued_pass():
    """call N queues the pass for stack B (next_stack=B); call N+1
    on B fails its argument checks (in C); the caller refills B with other
    images; call N+2 on B must compute its own histograms -- not take the
    queued ones of B's old contents."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W = 480, 640
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    sa, ta = synth.render_stack(rig, seed=21, view_deg=0.0, device="cuda")
    sb, tb = synth.render_stack(rig, seed=22, view_deg=30.0, device="cuda")
    sc, tc = synth.render_stack(rig, seed=23, view_deg=60.0, device="cuda")
    sc[1].add_(40)  # a brighter black plane: other thresholds than B's
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    kw = dict(maps=True, cloud=True, xyz_dtype=torch.float32)
    ref_c = _snap(eng.decode_triangulate(sc, texture=tc, out={}, **kw), eng)
    eng.sync()
    ref_b = _snap(eng.decode_triangulate(sb, texture=tb, out={}, **kw), eng)
    eng.sync()
    assert not np.array_equal(ref_b[-1], ref_c[-1]), "the test needs B and C to have other thresholds"
    B, TB = sb.clone(), tb.clone()
    eng.decode_triangulate(sa, texture=ta, out={}, next_stack=B, **kw)
    with pytest.raises(ValueError):
        eng.decode_triangulate(B, 70000, texture=TB, out={}, **kw)  # n_cols > 65536: EINVAL in C
    eng.sync()
    B.copy_(sc)
    TB.copy_(tc)
    r = eng.decode_triangulate(B, texture=TB, out={}, **kw)
    eng.sync()
    _same(_snap(r, eng), ref_c, "refilled B after a failed chained call")


def test_failed_arming_leaves_counts_alone():
    """mask_counts plus a bad next_stack raises before anything is
    armed; the next plain call leaves that counts tensor untouched (and a
    C-side failure consumes an armed counts pointer too)."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W = 96, 128
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    st, tx = synth.render_stack(rig, seed=2, device="cuda")
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    counts = torch.full((1,), -7, dtype=torch.int64, device="cuda")
    flat = torch.empty(st.numel() + 1, dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        eng.decode_triangulate(st, texture=tx, mask_counts=counts, next_stack=flat[1:].view(st.shape))
    eng.decode_triangulate(st, texture=tx)
    eng.sync()
    assert counts.item() == -7
    with pytest.raises(ValueError):
        eng.decode_triangulate(st, 70000, texture=tx, mask_counts=counts)
    eng.decode_triangulate(st, texture=tx)
    eng.sync()
    assert counts.item() == -7
    good = torch.zeros(1, dtype=torch.int64, device="cuda")
    r = eng.decode_triangulate(st, texture=tx, maps=True, mask_counts=good)
    eng.sync()
    assert good.item() == int(r["mask"].sum().item())


def test_prepared_call_after_close_raises():
    """Reconstructor.close() closes its prepared calls; running one
    afterwards raises instead of touching a freed context."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W = 96, 128
    rig = synth.Rig(H=H, W=W)
    cal = synth.make_calibration(rig)
    st, tx = synth.render_stack(rig, seed=3, device="cuda")
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    pc = eng.prepare(st, texture=tx, cloud=True, out={})
    pc.run()
    eng.sync()
    eng.close()
    with pytest.raises(RuntimeError):
        pc.run()


def test_decode_dynamic_grid_equals_strided():
    """The dynamic decode grid (cloud-only calls: k_decode's chunk groups after
    the first round pulled from per-view counters in the super-block buffer,
    which k_cloud zeroes) against the strided grid of a maps call: identical
    clouds, chained (pre-stats) and not, on 1080p views whose chunk groups
    outnumber the capped grid; sl_time_kernels re-runs the dynamic k_decode on
    fresh counters (a full decode each time)."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W, V = 1080, 1920, 3
    rig, base, A, TA = _group_views(H, W, V, True, 500)
    cal = synth.make_calibration(rig, with_Nc=False)
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    ref = _snap(eng.decode_triangulate(A, out={}, texture=TA, maps=True, cloud=True, xyz_dtype=torch.float32),
                eng)[:3]
    eng.sync()
    t_ref = eng.time_kernels(5)
    for k in range(3):
        r = eng.decode_triangulate(A, out={}, texture=TA, maps=False, cloud=True, xyz_dtype=torch.float32,
                                   next_stack=A if k < 2 else None)
        eng.sync()
        _same(_snap(r, eng)[:3], ref, f"dynamic call {k}")
    t_dyn = eng.time_kernels(5)
    assert t_dyn[0] > 0.3 * t_ref[0], (t_dyn, t_ref)
    r = eng.decode_triangulate(A, out={}, texture=TA, maps=False, cloud=True, xyz_dtype=torch.float32)
    eng.sync()
    _same(_snap(r, eng)[:3], ref, "after the re-runs")


@pytest.mark.parametrize("frame", ["decide", "3k_unaligned", "3k_wide_projector"])
def test_graphs_replay_in_any_phase(frame):
    """Phase safety: graphs of 1, 3 and 5 chained
    calls over three views (odd launch-group counts, their last call queuing a
    pass for a stack the graph's first call does not decode), each replayed
    several times, interleaved with one another, with eager chained calls
    (whose queued pass a replay must not disturb) and with sl_time_kernels:
    every call's maps, mask, thresholds and cloud bit-identical to the same
    call made alone, and one view to the oracle.  On the decide path (aligned
    640x480 frames) and on the 3-kernel path (k_count's histogram
    release over its waves and its super_produce under replay) -- an
    unaligned 500x360 frame (W % 16 != 0) and a 2560-column projector (Wp >
    2048, whose aligned calls still queue pre-stats passes the 3-kernel path
    never takes: they must be cleared before k_decode accumulates)."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W, Wp, Hp = {"decide": (480, 640, 1920, 1080), "3k_unaligned": (360, 500, 1920, 1080),
                    "3k_wide_projector": (480, 640, 2560, 1080)}[frame]
    rig = synth.Rig(H=H, W=W, Wp=Wp, Hp=Hp)
    cal = synth.make_calibration(rig)
    views = [synth.render_stack(rig, seed=140 + v, view_deg=30.0 * v, device="cuda") for v in range(3)]
    views[2][0][1].add_(25)  # a brighter black plane: other thresholds
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    kw = dict(maps=True, cloud=True, xyz_dtype=torch.float32)
    ref = []
    for st, tx in views:
        ref.append(_snap(eng.decode_triangulate(st, Wp, Hp, texture=tx, out={}, **kw), eng))
        eng.sync()
    assert eng.last_launch_info()[0] == (1 if frame == "decide" else 0)  # the kernel path under test
    assert not np.array_equal(ref[0][-1], ref[2][-1])
    s = torch.cuda.Stream()

    def call(i, o, nxt):
        st, tx = views[i]
        return eng.decode_triangulate(st, Wp, Hp, texture=tx, out=o, next_stack=views[nxt][0], **kw)

    graphs = {}
    for K in (1, 3, 5):
        seq = [(k + K) % 3 for k in range(K)]
        nxt = [(i + 1) % 3 for i in seq]  # the last call names a stack the first does not decode (K = 3 aside)
        outs = [{} for _ in range(K)]
        with torch.cuda.stream(s):
            for k in range(K):  # eager first: the outputs are allocated outside the capture
                call(seq[k], outs[k], nxt[k])
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            res = [call(seq[k], outs[k], nxt[k]) for k in range(K)]
        graphs[K] = (g, seq, res, outs)

    def replay(K, what):
        g, seq, res, outs = graphs[K]
        for o_ in outs:
            for v in o_.values():
                v.zero_()
        with torch.cuda.stream(s):
            g.replay()
        torch.cuda.synchronize()
        for k, r in enumerate(res):
            _same(_snap(r, eng)[:-1], ref[seq[k]][:-1], f"{what}: graph {K}, call {k}")

    def eager(i, nxt, what):
        with torch.cuda.stream(s):
            r = call(i, {}, nxt)
        torch.cuda.synchronize()
        _same(_snap(r, eng), ref[i], what)

    replay(5, "first replay")
    replay(1, "first replay")
    replay(1, "again")
    eager(0, 1, "eager 0 (queues a pass for 1)")
    replay(3, "between eager calls")
    replay(5, "between eager calls")
    eager(1, 2, "eager 1 takes its pass after two replays")
    replay(3, "again")
    eng.time_kernels(2)
    replay(5, "after re-runs")
    eager(2, 0, "eager after a replay")
    replay(1, "last")
    st, tx = views[2]
    col, row, mask, P, C = o.decode_triangulate(list(st.cpu().numpy()), tx.cpu().numpy(), cal, Wp, Hp)
    np.testing.assert_array_equal(ref[2][3][0], col)
    np.testing.assert_array_equal(ref[2][5][0], mask)
    np.testing.assert_array_equal(ref[2][0], P.astype(np.float32))


def test_reserve_then_capture_multi_group_call():
    """reserve() sizes every scratch buffer a captured call needs --
    the histograms of a whole launch group included -- so a call of two launch
    groups (34 1080p views: 32 + 2, the pass between its groups) captured right
    after reserve(), with no eager call first, allocates nothing and replays
    (twice) to the clouds of the same call made eagerly on another context."""
    from structured_light_for_3d_model_replication_amd import core, synth
    H, W, V = 1080, 1920, 34
    rig, base, A, TA = _group_views(H, W, V, False, 620)
    cal = synth.make_calibration(rig, with_Nc=False)
    kw = dict(texture=TA, maps=False, cloud=True, xyz_dtype=torch.float32)
    ref_eng = core.Reconstructor(torch.device("cuda", 0))
    ref_eng.set_calibration(cal, H, W)
    ref = _snap(ref_eng.decode_triangulate(A, out={}, **kw), ref_eng)[:3]
    ref_eng.sync()
    assert ref_eng.last_launch_info()[1] == 2
    ref_eng.close()
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(cal, H, W)
    eng.reserve(V, H * W)
    out = {"xyz": torch.empty((V * H * W, 3), dtype=torch.float32, device="cuda"),
           "bgr": torch.empty((V * H * W, 3), dtype=torch.uint8, device="cuda"),
           "view_offsets": torch.empty(V + 1, dtype=torch.int64, device="cuda")}
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
        r = eng.decode_triangulate(A, out=out, **kw)
    for rep in range(2):
        out["xyz"].zero_()
        with torch.cuda.stream(s):
            g.replay()
        torch.cuda.synchronize()
        _same(_snap(r, eng)[:3], ref, f"replay {rep}")
