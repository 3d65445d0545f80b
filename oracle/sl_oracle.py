"""CPU oracle for the Gray-code decode + ray/plane triangulation path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this module;
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg use it, and only as the checker / the timed CPU baseline.

This is a NumPy restatement of the reference algorithm, written so that every
floating-point and integer operation happens in the same order and dtype as the
reference, which makes it bit-exact against the reference's outputs:

* ``gray_decode_images``   <- server/sl_system.py:508-580 (adaptive mask) and
                              multi_point_cloud_process.py:23-71 /
                              Old/process_cloud.py:25-107 (fixed mask)
* ``reconstruct_point_cloud`` <- server/sl_system.py:584-653
                              (== multi_point_cloud_process.py:73-119)
* ``ply_text``             <- server/sl_system.py:665-691
                              (== multi_point_cloud_process.py:121-131)
* ``apply_pose``           <- not in the reference hot path; the turntable pose
                              epilogue of BASELINE config 5 (f64, fixed order).

Parity pin: ``tests/golden/*.npz`` were produced by running the reference's own
functions (see ``tests/golden/make_golden.py``); ``tests/test_oracle_golden.py``
checks this module against every one of them bit for bit.
"""
from __future__ import annotations

import numpy as np

MASK_ADAPTIVE = "adaptive"   # sl_system.py:526-535
MASK_FIXED = "fixed"         # multi_point_cloud_process.py:36-38


def n_bits(n: int) -> int:
    """int(np.ceil(np.log2(n))) as at sl_system.py:538-539."""
    return int(np.ceil(np.log2(n)))


def check_stack_length(n_files: int, n_cols: int, n_rows: int) -> None:
    """Raise the errors the reference raises for a stack of ``n_files`` images.

    sl_system.py:515-516 raises ValueError below 4 files.  decode_sequence
    (sl_system.py:549-554) reads pairs while ``current_idx < len(files)`` and
    indexes ``files[current_idx + 1]`` unguarded, so an odd dangling file that is
    reached raises IndexError.
    """
    if n_files < 4:
        raise ValueError("Not enough images in folder to decode.")
    idx = 2
    for _ in range(n_bits(n_cols) + n_bits(n_rows)):
        if idx >= n_files:
            break
        if idx + 1 >= n_files:
            raise IndexError("list index out of range")
        idx += 2


def _decode_sequence(images, start: int, nbits: int):
    """decode_sequence, sl_system.py:544-572 (shared running file index)."""
    h, w = images[0].shape
    gray_val = np.zeros((h, w), dtype=np.int32)
    idx = start
    for b in range(nbits):
        if idx >= len(images):
            break
        p = images[idx].astype(np.float32)
        i = images[idx + 1].astype(np.float32)
        idx += 2
        bit = np.zeros((h, w), dtype=np.int32)
        bit[p > i] = 1
        gray_val = np.bitwise_or(gray_val, np.left_shift(bit, nbits - 1 - b))
    # Gray -> binary: repeated xor with right shifts until every pixel's shifted
    # value is zero (sl_system.py:567-570).
    m = np.right_shift(gray_val, 1)
    while np.any(m > 0):
        gray_val = np.bitwise_xor(gray_val, m)
        m = np.right_shift(m, 1)
    return gray_val, idx


def valid_mask(white_u8, black_u8, mask_mode: str = MASK_ADAPTIVE):
    """Shadow / contrast mask.

    adaptive: sl_system.py:519-535 -- float32 contrast, np.percentile(black, 95)
    and max(contrast), float32 thresholds.
    fixed:    multi_point_cloud_process.py:31-38 -- white > 40 and contrast > 10.
    """
    white = white_u8.astype(np.float32)
    black = black_u8.astype(np.float32)
    if mask_mode == MASK_ADAPTIVE:
        contrast = white - black
        noise_floor = np.percentile(black, 95)
        dynamic_range = np.max(contrast)
        return (white > (noise_floor * 1.5)) & (contrast > (dynamic_range * 0.05))
    if mask_mode == MASK_FIXED:
        return (white > 40) & ((white - black) > 10)
    raise ValueError(f"unknown mask_mode {mask_mode!r}")


def adaptive_thresholds(white_u8, black_u8):
    """(noise_floor, dynamic_range) as float32, exactly as sl_system.py:526-528."""
    white = white_u8.astype(np.float32)
    black = black_u8.astype(np.float32)
    return np.percentile(black, 95), np.max(white - black)


def gray_decode_images(images, n_cols: int = 1920, n_rows: int = 1080,
                       mask_mode: str = MASK_ADAPTIVE):
    """gray_decode on an in-memory image list (sorted-file order).

    Returns (col_map int32, row_map int32, valid_mask bool); the texture is a
    separate colour read of file 0 in the reference (sl_system.py:580).
    """
    images = [np.asarray(im) for im in images]
    check_stack_length(len(images), n_cols, n_rows)
    mask = valid_mask(images[0], images[1], mask_mode)
    col_map, idx = _decode_sequence(images, 2, n_bits(n_cols))
    row_map, _ = _decode_sequence(images, idx, n_bits(n_rows))
    return col_map, row_map, mask


def pinhole_rays(valid_indices, h: int, w: int, cam_K):
    """Camera rays regenerated from K (sl_system.py:607-621)."""
    fx, fy = cam_K[0, 0], cam_K[1, 1]
    cx, cy = cam_K[0, 2], cam_K[1, 2]
    y_v, x_v = np.unravel_index(valid_indices, (h, w))
    x_n = (x_v - cx) / fx
    y_n = (y_v - cy) / fy
    z_n = np.ones_like(x_n)
    rays = np.stack((x_n, y_n, z_n))
    rays /= np.linalg.norm(rays, axis=0)
    return rays


def numerator_fixed(n, Oc):
    """n.Oc for each column of n (3, M) in the order libslgpu.so fixes:
    fma(n2, o2, fma(n0, o0, fl(n1 o1))) -- the order of the transposed
    OpenBLAS dgemv np.dot runs for the reference's strided N.T
    (sl_system.py:629-639) on the build host.  Exact rational arithmetic per
    distinct plane, correctly rounded to f64 at each step."""
    from fractions import Fraction as F
    o = [float(v) for v in np.asarray(Oc, dtype=np.float64).reshape(3)]
    cols = np.ascontiguousarray(n.T)
    uniq, inv = np.unique(cols, axis=0, return_inverse=True)
    vals = np.empty(len(uniq))
    for i, (n0, n1, n2) in enumerate(uniq.tolist()):
        p1 = float(F(n1) * F(o[1]))
        f = float(F(n0) * F(o[0]) + F(p1))
        vals[i] = float(F(n2) * F(o[2]) + F(f))
    return vals[np.asarray(inv).reshape(-1)]


def reconstruct_point_cloud(col_map, row_map, mask, texture, calib, oc_dot="blas"):
    """Ray/plane triangulation, sl_system.py:584-653.

    Returns (P float64 (N,3), C uint8 (N,3) BGR) in ascending pixel order.
    ``row_map`` is accepted and unused, as in the reference.  ``oc_dot``:
    "blas" computes n.Oc with np.dot as the reference does (:639) -- its
    rounding follows the host's BLAS kernel, so it is host dependent when
    Oc != 0; "fixed" uses the order of ``numerator_fixed``.
    """
    del row_map
    Nc = np.asarray(calib["Nc"])
    Oc = np.asarray(calib["Oc"])
    planes = np.asarray(calib["wPlaneCol"])
    if planes.shape[0] == 4:
        planes = planes.T
    h, w = col_map.shape
    col_flat = col_map.flatten()
    tex_flat = texture.reshape(-1, 3)
    idx = np.where(mask.flatten())[0]
    if Nc.ndim == 2 and Nc.shape[1] == h * w:
        rays = Nc[:, idx]
    else:
        rays = pinhole_rays(idx, h, w, np.asarray(calib["cam_K"]))
    cols = np.clip(col_flat[idx], 0, planes.shape[0] - 1)
    pl = planes[cols, :]
    n = pl[:, 0:3].T
    d = pl[:, 3]
    denom = np.sum(n * rays, axis=0)
    if oc_dot == "fixed":
        numer = numerator_fixed(n, Oc) + d
    else:
        numer = np.dot(n.T, Oc).flatten() + d
    ok = np.abs(denom) > 1e-6
    t = -numer[ok] / denom[ok]
    P = Oc + rays[:, ok] * t
    return P.T, tex_flat[idx[ok]]


def apply_pose(points, pose):
    """Turntable pose epilogue (config 5): p' = R p + t in f64, row order
    ((m0*x + m1*y) + m2*z) + m3 -- the order the HIP epilogue uses."""
    M = np.asarray(pose, dtype=np.float64).reshape(4, 4)
    x, y, z = points[:, 0], points[:, 1], points[:, 2]
    out = np.empty_like(points)
    for r in range(3):
        out[:, r] = ((M[r, 0] * x + M[r, 1] * y) + M[r, 2] * z) + M[r, 3]
    return out


def decode_triangulate(images, texture, calib, n_cols=1920, n_rows=1080,
                       mask_mode=MASK_ADAPTIVE, pose=None, oc_dot="blas"):
    """gray_decode + reconstruct_point_cloud in one call (generate_cloud body,
    sl_system.py:658-661).  ``texture`` is BGR (H,W,3); None -> file 0
    replicated (what cv2.imread colour returns for a single-channel file)."""
    col_map, row_map, mask = gray_decode_images(images, n_cols, n_rows, mask_mode)
    if texture is None:
        texture = np.repeat(np.asarray(images[0])[:, :, None], 3, axis=2)
    P, C = reconstruct_point_cloud(col_map, row_map, mask, texture, calib, oc_dot)
    if pose is not None:
        P = apply_pose(P, pose)
    return col_map, row_map, mask, P, C


def ply_text(points, colors) -> str:
    """ASCII PLY exactly as sl_system.py:671-691 writes it (xyz %.4f, RGB)."""
    out = ["ply\n", "format ascii 1.0\n", f"element vertex {len(points)}\n",
           "property float x\n", "property float y\n", "property float z\n",
           "property uchar red\n", "property uchar green\n", "property uchar blue\n",
           "end_header\n"]
    for p, c in zip(points, colors):
        out.append(f"{p[0]:.4f} {p[1]:.4f} {p[2]:.4f} {c[2]} {c[1]} {c[0]}\n")
    return "".join(out)
