"""The PLY text formatted on the GPU (sl_write_ply_device, ply.save_ply_device)
is byte-identical to the host formatter (ply.ply_text), whose bytes are pinned
against the reference's own PLY files and CPython's %.4f (tests/test_ply_io.py):
random and edge values in f64 and f32 (ties, signed zeros, tiny and 8.99e11
magnitudes, every colour width), the empty cloud, and clouds the device hands
back to the host (NaN, inf, |x| >= 9e11: libc's %.4f)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _edge_values():
    v = [0.0, -0.0, 0.00005, -0.00005, 0.00015, 0.00025, 1.23445, 1.23455, 0.5, -0.5, 1e-300, -1e-300, 5e-324,
         123456.78905, 8.99e11, -8.99e11, 899999999999.99994, 2.0 ** -30, 1.0 / 3.0, -2.0 / 3.0, 9.99995, 99.99995]
    # exact ties at the 5th decimal: k / 2^... with a binary-exact .xxxx5
    v += [(2 * k + 1) / 2.0 ** 5 for k in range(-40, 40)]
    return np.array(v, dtype=np.float64)


def _check(tmp_path, xyz, bgr, name):
    from structured_light_for_3d_model_replication_amd import ply
    want = ply.ply_text(xyz, bgr).encode()
    out = tmp_path / f"{name}.ply"
    ply.save_ply_device(torch.from_numpy(xyz).cuda(), torch.from_numpy(bgr).cuda(), str(out))
    got = out.read_bytes()
    assert got == want, (name, len(got), len(want))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_device_ply_matches_host_formatter(tmp_path, dtype):
    rng = np.random.default_rng(17)
    n = 300_017  # many workgroups, a ragged last one
    xyz = (rng.standard_normal((n, 3)) * rng.choice([1e-3, 1.0, 300.0, 1e6], size=(n, 1))).astype(dtype)
    e = _edge_values().astype(dtype)
    xyz[: len(e), 0] = e
    xyz[: len(e), 1] = -e[::-1]
    xyz[: len(e), 2] = e * 3
    bgr = rng.integers(0, 256, (n, 3), dtype=np.uint8)
    bgr[:6] = [[0, 9, 10], [99, 100, 255], [255, 255, 255], [0, 0, 0], [10, 100, 1], [5, 50, 250]]
    _check(tmp_path, xyz, bgr, f"rand_{np.dtype(dtype).name}")


def test_device_ply_empty_and_single(tmp_path):
    _check(tmp_path, np.zeros((0, 3), np.float64), np.zeros((0, 3), np.uint8), "empty")
    _check(tmp_path, np.array([[1.5, -2.25, 3.0]]), np.array([[1, 2, 3]], np.uint8), "one")


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf, 9.5e11, -3e15])
def test_device_ply_hands_libc_values_back_to_the_host(tmp_path, bad):
    rng = np.random.default_rng(5)
    xyz = rng.standard_normal((5000, 3))
    xyz[1234, 1] = bad
    bgr = rng.integers(0, 256, (5000, 3), dtype=np.uint8)
    _check(tmp_path, xyz, bgr, "fallback")


def test_device_ply_of_a_decoded_cloud(tmp_path):
    """A real cloud straight from decode_triangulate's outputs (f64 and f32
    xyz, device tensors, never copied to the host by the caller)."""
    from structured_light_for_3d_model_replication_amd import core, ply, synth
    rig = synth.Rig(H=240, W=320)
    stack, tex = synth.render_stack(rig, seed=9, device="cuda")
    eng = core.Reconstructor(torch.device("cuda", 0))
    eng.set_calibration(synth.make_calibration(rig), rig.H, rig.W)
    for dt in (torch.float64, torch.float32):
        cl = eng.decode_triangulate(stack, texture=tex, cloud=True, xyz_dtype=dt)["cloud"]
        eng.sync()
        n = cl.total()
        assert n > 1000
        out = tmp_path / "cloud.ply"
        ply.save_ply_device(cl.xyz[:n], cl.bgr[:n], str(out))
        assert out.read_bytes() == ply.ply_text(cl.xyz[:n].cpu().numpy(), cl.bgr[:n].cpu().numpy()).encode()
    eng.close()


def test_device_ply_replaces_an_existing_file(tmp_path):
    """A re-run over the same scan: the PLY already there (large, so the
    writer renames it away and unlinks it beside the write) is replaced by
    the same bytes a new file gets, its mode kept, no side file left."""
    import os
    import stat
    import time
    from structured_light_for_3d_model_replication_amd import ply
    rng = np.random.default_rng(21)
    xyz = rng.standard_normal((50_000, 3)) * 50
    bgr = rng.integers(0, 256, (50_000, 3), dtype=np.uint8)
    out = tmp_path / "scan.ply"
    out.write_bytes(b"z" * (24 << 20))
    os.chmod(out, 0o600)
    ply.save_ply_device(torch.from_numpy(xyz).cuda(), torch.from_numpy(bgr).cuda(), str(out))
    assert out.read_bytes() == ply.ply_text(xyz, bgr).encode()
    assert stat.S_IMODE(os.stat(out).st_mode) == 0o600
    for _ in range(100):
        if [p.name for p in tmp_path.iterdir()] == ["scan.ply"]:
            break
        time.sleep(0.05)
    assert [p.name for p in tmp_path.iterdir()] == ["scan.ply"]
