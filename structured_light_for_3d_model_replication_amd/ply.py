"""ASCII PLY writer, byte-identical to the reference's.

Format of server/sl_system.py:671-691 (== multi_point_cloud_process.py:121-131,
Old/process_cloud.py:200-219): ASCII header, then per point
``"%.4f %.4f %.4f %d %d %d\\n"`` with the colour swapped from BGR to RGB.

The reference formats one point per Python f-string (~0.3 Mpt/s).  Here whole
chunks are formatted with one ``%`` operation on a flat tuple; ``%.4f`` and
``f"{x:.4f}"`` both use CPython's correctly rounded ``PyOS_double_to_string``,
so the bytes are identical.
"""
from __future__ import annotations

import numpy as np

_HEADER = ("ply\nformat ascii 1.0\nelement vertex {n}\nproperty float x\nproperty float y\n"
           "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")
_CHUNK = 1 << 16


def ply_chunks(points, colors):
    """Yield the PLY text in pieces (header first)."""
    points = np.asarray(points, dtype=np.float64)
    colors = np.asarray(colors)
    n = len(points)
    if len(colors) != n:
        raise ValueError("points and colors differ in length")
    yield _HEADER.format(n=n)
    line = "%.4f %.4f %.4f %d %d %d\n"
    for s in range(0, n, _CHUNK):
        p = points[s:s + _CHUNK]
        c = colors[s:s + _CHUNK].astype(np.int64)
        m = len(p)
        flat = np.empty((m, 6), dtype=object)
        flat[:, 0:3] = p.tolist() if m else np.empty((0, 3))
        flat[:, 3] = c[:, 2].tolist()
        flat[:, 4] = c[:, 1].tolist()
        flat[:, 5] = c[:, 0].tolist()
        yield (line * m) % tuple(flat.ravel().tolist())


def ply_text(points, colors) -> str:
    return "".join(ply_chunks(points, colors))


def save_ply(points, colors, filename) -> None:
    """save_ply(points, colors, filename) of multi_point_cloud_process.py:121."""
    with open(filename, "w") as f:
        for piece in ply_chunks(points, colors):
            f.write(piece)
