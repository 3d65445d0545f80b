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
import threading

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


def save_ply(points, colors, filename, binary: bool = False) -> None:
    """save_ply(points, colors, filename) of multi_point_cloud_process.py:121.

    ``binary=True`` writes binary_little_endian with the same properties
    (float32 xyz, uchar RGB): what Open3D's write_point_cloud writes by default.
    """
    P, C, n, dt = _arrays(points, colors)
    fn = _lib.load().sl_write_ply_binary if binary else _lib.load().sl_write_ply
    _lib.check(fn(os.fsencode(filename), P.ctypes.data, dt, C.ctypes.data, n, _THREADS), None,
               f"cannot write {filename}")


_WRITERS: dict = {}  # device -> a context of its own for device-side PLY formatting (its scratch, its lock)
_WRITERS_LOCK = threading.Lock()


def save_ply_device(xyz, bgr, filename, stream=None) -> None:
    """save_ply of a cloud in GPU memory (torch tensors: xyz (n, 3) float32 /
    float64, bgr (n, 3) uint8): the text is formatted on the GPU by the same
    digit code as the host formatter (one thread per point), copied back in
    chunks and written -- byte-identical to save_ply(xyz.cpu(), bgr.cpu(),
    filename), without the points' D2H or any host formatting.  A context of
    its own per device keeps the writer off the decoding contexts' locks."""
    from . import core
    with _WRITERS_LOCK:
        key = str(xyz.device)
        if key not in _WRITERS:
            _WRITERS[key] = core.Reconstructor(xyz.device)
        w = _WRITERS[key]
    w.write_ply(filename, xyz, bgr, stream)


def save_ply_open3d(points, colors, filename, normals=None, binary: bool = True) -> None:
    """The file o3d.io.write_point_cloud writes for a cloud with points,
    optional normals and colours (processing.py:181): binary little-endian
    (``binary=False``: ASCII) with ``comment Created by Open3D``, double x y z,
    double nx ny nz, uchar red green blue.  ``colors`` are BGR uint8 (written
    as RGB).  Layout restated from Open3D's FilePLY.cpp; unpinned (no Open3D
    in this image)."""
    P = np.ascontiguousarray(np.asarray(points, dtype=np.float64)).reshape(-1, 3)
    C = np.ascontiguousarray(np.asarray(colors, dtype=np.uint8)).reshape(-1, 3)
    n = len(P)
    if len(C) != n or (normals is not None and len(normals) != n):
        raise ValueError("points, colors and normals differ in length")
    fields = [("x", "<f8"), ("y", "<f8"), ("z", "<f8")]
    if normals is not None:
        fields += [("nx", "<f8"), ("ny", "<f8"), ("nz", "<f8")]
    fields += [("red", "u1"), ("green", "u1"), ("blue", "u1")]
    rec = np.empty(n, dtype=np.dtype(fields))
    rec["x"], rec["y"], rec["z"] = P[:, 0], P[:, 1], P[:, 2]
    if normals is not None:
        Nn = np.asarray(normals, dtype=np.float64).reshape(-1, 3)
        rec["nx"], rec["ny"], rec["nz"] = Nn[:, 0], Nn[:, 1], Nn[:, 2]
    rec["red"], rec["green"], rec["blue"] = C[:, 2], C[:, 1], C[:, 0]
    tnames = {"<f8": "double", "u1": "uchar"}
    head = ["ply", f"format {'binary_little_endian' if binary else 'ascii'} 1.0", "comment Created by Open3D",
            f"element vertex {n}"] + [f"property {tnames[t]} {nm}" for nm, t in fields] + ["end_header", ""]
    with open(filename, "wb") as f:
        f.write("\n".join(head).encode("ascii"))
        if binary:
            rec.tofile(f)
        else:
            # rply's ASCII writer: "%g" for doubles, "%d" for uchar, space-separated
            cols = [rec[nm] for nm, _ in fields]
            for i in range(n):
                f.write((" ".join(f"{float(c[i]):g}" if c.dtype.kind == "f" else str(int(c[i])) for c in cols)
                         + "\n").encode("ascii"))


_PLY_TYPES = {"float": "<f4", "float32": "<f4", "double": "<f8", "float64": "<f8", "uchar": "u1",
              "uint8": "u1", "char": "i1", "int8": "i1", "short": "<i2", "int16": "<i2", "ushort": "<u2",
              "uint16": "<u2", "int": "<i4", "int32": "<i4", "uint": "<u4", "uint32": "<u4"}


def read_normals(filename):
    """nx ny nz of a vertex-only PLY (float64 (N,3)), or None when absent."""
    cols = _read_columns(filename)
    if not all(c in cols for c in ("nx", "ny", "nz")):
        return None
    return np.stack([cols["nx"], cols["ny"], cols["nz"]], 1).astype(np.float64)


def _read_columns(filename):
    """{property: column} of a vertex-only PLY (ASCII or binary_little_endian)."""
    with open(filename, "rb") as f:
        data = f.read()
    end = data.find(b"end_header\n")
    if not data.startswith(b"ply") or end < 0:
        raise ValueError(f"{filename}: not a PLY file")
    head = data[:end].decode("ascii").split("\n")
    fmt, n, props = None, 0, []
    for line in head:
        t = line.split()
        if not t:
            continue
        if t[0] == "format":
            fmt = t[1]
        elif t[0] == "element":
            if t[1] != "vertex":
                raise ValueError(f"{filename}: only vertex elements are supported")
            n = int(t[2])
        elif t[0] == "property":
            if t[1] == "list":
                raise ValueError(f"{filename}: list properties are not supported")
            props.append((t[2], _PLY_TYPES[t[1]]))
    body = data[end + len(b"end_header\n"):]
    names = [p for p, _ in props]
    if fmt == "ascii":
        rows = np.loadtxt(body.decode("ascii").splitlines(), dtype=np.float64, ndmin=2) if n else \
            np.zeros((0, len(props)))
        cols = {p: rows[:, i] for i, p in enumerate(names)}
    elif fmt == "binary_little_endian":
        rec = np.frombuffer(body, dtype=np.dtype(props), count=n)
        cols = {p: rec[p] for p in names}
    else:
        raise ValueError(f"{filename}: unsupported format {fmt}")
    return cols


def read_ply(filename):
    """-> (points float64 (N,3), colors uint8 (N,3) BGR) of a vertex-only PLY
    (ASCII or binary_little_endian), as o3d.io.read_point_cloud feeds
    processing.py:116-182.  Colour is swapped back to BGR, the reference's
    in-memory order; a file without colour gives zeros."""
    cols = _read_columns(filename)
    n = len(cols["x"])
    P = np.stack([cols["x"], cols["y"], cols["z"]], 1).astype(np.float64)
    if all(c in cols for c in ("red", "green", "blue")):
        C = np.stack([cols["blue"], cols["green"], cols["red"]], 1).astype(np.uint8)
    else:
        C = np.zeros((n, 3), np.uint8)
    return P, C
