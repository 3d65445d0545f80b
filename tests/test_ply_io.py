"""PLY writer and stack ingest (host side)."""
import os

import numpy as np
import pytest
from PIL import Image

from structured_light_for_3d_model_replication_amd import io, ply
from tests import golden_io as g


@pytest.mark.parametrize("name", ["sl_generate_cloud_e2e", "mp_fixed_mask"])
def test_ply_byte_identical_to_reference_writer(name, tmp_path):
    d = g.load(name)
    out = tmp_path / "x.ply"
    ply.save_ply(d["P"], d["C"], out)
    assert out.read_text() == g.ply_text(d["meta"]["ply"])


def test_ply_edge_values():
    P = np.array([[0.0, -0.0, 1e-5], [-1.23455, 2.00005, 1e6], [123.45675, -0.00005, 3.5]])
    C = np.array([[1, 2, 3], [255, 0, 128], [7, 8, 9]], dtype=np.uint8)
    expect = "".join(f"{p[0]:.4f} {p[1]:.4f} {p[2]:.4f} {c[2]} {c[1]} {c[0]}\n" for p, c in zip(P, C))
    assert ply.ply_text(P, C).endswith(expect)
    assert ply.ply_text(np.zeros((0, 3)), np.zeros((0, 3), np.uint8)).endswith("end_header\n")


def test_read_stack_order_and_errors(tmp_path):
    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 256, (6, 9), dtype=np.uint8) for _ in range(6)]
    for i, im in enumerate(imgs):
        Image.fromarray(im).save(tmp_path / f"{i + 1:02d}.png")
    Image.fromarray(np.zeros((6, 9, 3), np.uint8)).save(tmp_path / "zz.jpg")  # ignored
    st, tex, files = io.read_stack(str(tmp_path))
    assert [os.path.basename(f) for f in files] == [f"{i + 1:02d}.png" for i in range(6)]
    np.testing.assert_array_equal(st, np.stack(imgs))
    np.testing.assert_array_equal(tex, np.repeat(imgs[0][:, :, None], 3, axis=2))
    # .bmp takes precedence over .png (sl_system.py:510-512)
    for i in range(4):
        Image.fromarray(imgs[i]).save(tmp_path / f"b{i}.bmp")
    st2, _, files2 = io.read_stack(str(tmp_path))
    assert all(f.endswith(".bmp") for f in files2) and st2.shape[0] == 4
    empty = tmp_path / "empty"
    empty.mkdir()
    with pytest.raises(ValueError):
        io.read_stack(str(empty))


def test_colour_conversion_matches_opencv_weights(tmp_path):
    rgb = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [10, 20, 30]]], dtype=np.uint8)
    Image.fromarray(rgb).save(tmp_path / "c.png")
    gray = io.imread_gray(str(tmp_path / "c.png"))
    r, gch, b = rgb[..., 0].astype(int), rgb[..., 1].astype(int), rgb[..., 2].astype(int)
    np.testing.assert_array_equal(gray, (1868 * b + 9617 * gch + 4899 * r + 8192) >> 14)
    np.testing.assert_array_equal(io.imread_bgr(str(tmp_path / "c.png")), rgb[:, :, ::-1])


def _python_ply(P, C):
    """The reference's own formatting loop (sl_system.py:685-691), as text."""
    head = ("ply\nformat ascii 1.0\nelement vertex {}\nproperty float x\nproperty float y\nproperty float z\n"
            "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n").format(len(P))
    return head + "".join(f"{p[0]:.4f} {p[1]:.4f} {p[2]:.4f} {c[2]} {c[1]} {c[0]}\n"
                          for p, c in zip(P.tolist(), np.asarray(C).tolist()))


def test_native_formatter_matches_cpython_on_edge_values():
    rng = np.random.default_rng(5)
    ties = np.array([k + 0.5 for k in range(-20, 20)]) / 1e4  # not exact; plus exact binary ties below
    # x * 10^4 exactly k + 1/2 in binary (round-half-even decides), and near-ties
    exact_ties = np.array([1.03125, -1.03125, 1.0000305175781250, 0.0000305175781250, 3.00003125,
                           12.34565, 0.00025, 0.00015, -0.00005, 0.0])
    special = np.array([-0.0, 1e-320, -1e-320, 5e-324, 4.9999e-5, 5.0001e-5, -4.9999e-5, 1e15, -1e15,
                        123456789012.3456, 9.0e11, 8.99999999999e11, 1.7976931348623157e308, -1e300,
                        np.inf, -np.inf, np.nan, 2.0 ** 53 / 1e4, 2.0 ** 60, 0.99995, 0.99994999, 9.99995])
    rnd = np.concatenate([rng.normal(0, 500, 20000), rng.uniform(-1, 1, 20000) * 1e-3,
                          np.round(rng.normal(0, 100, 20000), 5), rng.normal(0, 1e8, 2000)])
    vals = np.concatenate([ties, exact_ties, special, rnd])
    vals = vals[: (len(vals) // 3) * 3]
    P = vals.reshape(-1, 3)
    C = rng.integers(0, 256, P.shape, dtype=np.uint8)
    assert ply.ply_text(P, C) == _python_ply(P, C)
    # float32 points are formatted as their exact float64 value (numpy upcast)
    with np.errstate(over="ignore"):
        P32 = P.astype(np.float32)
    assert ply.ply_text(P32, C) == _python_ply(P32.astype(np.float64), C)


def test_native_writer_multithreaded_large(tmp_path):
    rng = np.random.default_rng(6)
    P = rng.normal(0, 300, (300_000, 3))
    C = rng.integers(0, 256, P.shape, dtype=np.uint8)
    f = tmp_path / "big.ply"
    ply.save_ply(P, C, str(f))
    assert f.read_text() == _python_ply(P, C)
    with pytest.raises(OSError):
        ply.save_ply(P[:3], C[:3], str(tmp_path / "no_such_dir" / "x.ply"))


def test_binary_ply_layout_and_roundtrip(tmp_path):
    """Binary PLY: the reference header's properties as binary_little_endian,
    15-byte records (float32 xyz, RGB); read_ply gives back (P, C BGR)."""
    rng = np.random.default_rng(7)
    P = rng.normal(0, 300, (200_003, 3))
    C = rng.integers(0, 256, P.shape, dtype=np.uint8)
    f = tmp_path / "b.ply"
    ply.save_ply(P, C, str(f), binary=True)
    raw = f.read_bytes()
    head = (b"ply\nformat binary_little_endian 1.0\nelement vertex 200003\nproperty float x\n"
            b"property float y\nproperty float z\nproperty uchar red\nproperty uchar green\n"
            b"property uchar blue\nend_header\n")
    assert raw.startswith(head) and len(raw) == len(head) + 15 * len(P)
    rec = np.frombuffer(raw[len(head):], dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"),
                                                ("r", "u1"), ("g", "u1"), ("b", "u1")])
    np.testing.assert_array_equal(np.stack([rec["x"], rec["y"], rec["z"]], 1), P.astype(np.float32))
    np.testing.assert_array_equal(np.stack([rec["b"], rec["g"], rec["r"]], 1), C)
    P2, C2 = ply.read_ply(str(f))
    np.testing.assert_array_equal(P2, P.astype(np.float32).astype(np.float64))
    np.testing.assert_array_equal(C2, C)
    ply.save_ply(P[:0], C[:0], str(f), binary=True)
    assert ply.read_ply(str(f))[0].shape == (0, 3)


@pytest.mark.parametrize("name", ["sl_generate_cloud_e2e", "mp_fixed_mask"])
def test_read_ply_ascii_reference_file(name, tmp_path):
    """read_ply on the reference's own ASCII PLY: %.4f values, BGR order back."""
    d = g.load(name)
    f = tmp_path / "r.ply"
    f.write_text(g.ply_text(d["meta"]["ply"]))
    P, C = ply.read_ply(str(f))
    expect = np.array([[float(f"{v:.4f}") for v in p] for p in d["P"]]).reshape(-1, 3)
    np.testing.assert_array_equal(P, expect)
    np.testing.assert_array_equal(C, d["C"])


def test_merge_file_orders(tmp_path):
    """processing.py:121 sorts the per-view clouds lexicographically;
    Old/new360Merge.py:7-20 by the first integer in the name."""
    from structured_light_for_3d_model_replication_amd import merge
    for n in ("view_100deg.ply", "view_10deg.ply", "view_20deg.ply", "view_0deg.ply", "notes.txt", "zz.PLY"):
        (tmp_path / n).write_text("")
    lex = [os.path.basename(f) for f in merge.ply_files(str(tmp_path))]
    num = [os.path.basename(f) for f in merge.ply_files(str(tmp_path), "numeric")]
    assert lex == ["view_0deg.ply", "view_100deg.ply", "view_10deg.ply", "view_20deg.ply"]
    assert num == ["view_0deg.ply", "zz.PLY", "view_10deg.ply", "view_20deg.ply", "view_100deg.ply"]
    with pytest.raises(ValueError):
        merge.ply_files(str(tmp_path), "mtime")


@pytest.mark.parametrize("binary", [True, False])
def test_open3d_layout_writer_round_trip(tmp_path, binary):
    """save_ply_open3d: the layout o3d.io.write_point_cloud writes for points +
    normals + colours (double x y z nx ny nz, uchar RGB); read back exactly
    (binary) / to %g (ASCII)."""
    rng = np.random.default_rng(2)
    P = rng.normal(size=(50, 3)) * 100
    N = rng.normal(size=(50, 3))
    C = rng.integers(0, 256, (50, 3), dtype=np.uint8)
    f = str(tmp_path / "o3d.ply")
    ply.save_ply_open3d(P, C, f, normals=N, binary=binary)
    head = open(f, "rb").read().split(b"end_header\n")[0].decode()
    assert "comment Created by Open3D" in head
    assert [ln.split()[-1] for ln in head.splitlines() if ln.startswith("property")] == \
        ["x", "y", "z", "nx", "ny", "nz", "red", "green", "blue"]
    P2, C2 = ply.read_ply(f)
    N2 = ply.read_normals(f)
    np.testing.assert_array_equal(C2, C)
    if binary:
        np.testing.assert_array_equal(P2, P)
        np.testing.assert_array_equal(N2, N)
    else:
        np.testing.assert_allclose(P2, P, rtol=1e-5)
        np.testing.assert_allclose(N2, N, rtol=1e-5, atol=1e-5)
    ply.save_ply_open3d(P, C, f)
    assert ply.read_normals(f) is None


def test_writer_replaces_large_files_and_keeps_links(tmp_path):
    """A large regular file already at the path (a re-run over the same scan)
    is replaced -- renamed away and unlinked beside the write -- with the
    same bytes as a fresh write and the old file's mode; no side file stays
    behind.  Symlinks are written through and hard-linked files truncated in
    place, as open(path, 'w') does."""
    import stat
    import time
    rng = np.random.default_rng(8)
    n = 200_000
    P = rng.standard_normal((n, 3)) * 100
    C = rng.integers(0, 256, (n, 3), dtype=np.uint8)
    want = ply.ply_text(P, C).encode()
    f = tmp_path / "scan.ply"
    f.write_bytes(b"x" * (20 << 20))
    os.chmod(f, 0o640)
    ply.save_ply(P, C, str(f))
    assert f.read_bytes() == want and stat.S_IMODE(os.stat(f).st_mode) == 0o640
    for _ in range(100):  # the old file's unlink runs on another thread
        if sorted(p.name for p in tmp_path.iterdir()) == ["scan.ply"]:
            break
        time.sleep(0.05)
    assert sorted(p.name for p in tmp_path.iterdir()) == ["scan.ply"]
    # a symlink: the target is written, the link stays a link
    tgt = tmp_path / "target.ply"
    tgt.write_bytes(b"y" * (20 << 20))
    lnk = tmp_path / "link.ply"
    lnk.symlink_to(tgt)
    ply.save_ply(P[:10], C[:10], str(lnk))
    assert lnk.is_symlink() and tgt.read_bytes() == ply.ply_text(P[:10], C[:10]).encode()
    # a hard-linked file: both names see the new bytes
    h2 = tmp_path / "hard2.ply"
    os.link(tgt, h2)
    ply.save_ply(P, C, str(tgt))
    assert h2.read_bytes() == want and os.stat(tgt).st_ino == os.stat(h2).st_ino
