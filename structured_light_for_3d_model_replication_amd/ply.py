"""ASCII PLY writer, byte-identical to the reference's.

Format of server/sl_system.py:671-691 (== multi_point_cloud_process.py:121-131,
Old/process_cloud.py:200-219): ASCII header, then per point
``"%.4f %.4f %.4f %d %d %d\\n"`` with the colour swapped from BGR to RGB.

The reference formats one point per Python f-string (~0.3 Mpt/s).  Here the
text is produced by libslgpu's host formatter (``sl_format_ply`` /
``sl_write_ply``): correctly rounded %.4f (ties to even, as CPython's
``PyOS_double_to_string``) from exact 128-bit integer arithmetic, on several
threads.  ``tests/test_ply_io.py`` pins the bytes against the reference's own
PLY output and against CPython's formatting on edge values.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib

_THREADS = max(1, min(16, os.cpu_count() or 1))


def _arrays(points, colors):
    P = np.asarray(points)
    if P.dtype not in (np.float32, np.float64):
        P = P.astype(np.float64)
    P = np.ascontiguousarray(P)
    C = np.ascontiguousarray(np.asarray(colors, dtype=np.uint8))
    n = len(P)
    if len(C) != n:
        raise ValueError("points and colors differ in length")
    if n and (P.shape[1:] != (3,) or C.shape[1:] != (3,)):
        raise ValueError("points and colors must be (N, 3)")
    return P, C, n, (_lib.SL_XYZ_F32 if P.dtype == np.float32 else _lib.SL_XYZ_F64)


def ply_text(points, colors) -> str:
    """The PLY file content as a str."""
    P, C, n, dt = _arrays(points, colors)
    L = _lib.load()
    ln = ctypes.c_int64()
    _lib.check(L.sl_format_ply(P.ctypes.data, dt, C.ctypes.data, n, _THREADS, None, 0, ctypes.byref(ln)),
               None, "sl_format_ply")
    buf = ctypes.create_string_buffer(ln.value)
    _lib.check(L.sl_format_ply(P.ctypes.data, dt, C.ctypes.data, n, _THREADS, buf, ln.value, ctypes.byref(ln)),
               None, "sl_format_ply")
    return buf.raw[: ln.value].decode("ascii")


def save_ply(points, colors, filename) -> None:
    """save_ply(points, colors, filename) of multi_point_cloud_process.py:121."""
    P, C, n, dt = _arrays(points, colors)
    _lib.check(_lib.load().sl_write_ply(os.fsencode(filename), P.ctypes.data, dt, C.ctypes.data, n, _THREADS),
               None, f"cannot write {filename}")
