"""CPU restatement of the calibration products of SLSystem.calibrate_final
(server/sl_system.py:348-403) -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker of the HIP kernels in
csrc/slcalib.hip; the product path (calibration.py) never calls it.

Pinned by tests/golden/calib_*.npz, which hold the reference's own
calibrate_final output (its OpenCV calls stubbed to return given K1, K2, R, T;
tests/golden/make_calib_golden.py).  The reference evaluates with NumPy 2.2.6
on OpenBLAS 0.3.29: its 3x3 @ 3x1 products, np.dot and the 1-D np.linalg.norm
(sqrt(dot(x, x))) are OpenBLAS kernels that accumulate left to right with fused
multiply-adds, fma(a2, b2, fma(a1, b1, a0*b0)) -- measured bit for bit in this
image over 3000 random cases; np.cross and the divisions are separate IEEE
operations.  The fma here is exact rational arithmetic rounded once.
"""
from __future__ import annotations

from fractions import Fraction

import numpy as np


def _fma(a: float, b: float, c: float) -> float:
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _dot3(a, b) -> float:
    """OpenBLAS 3-term dot / matmul row."""
    return _fma(a[2], b[2], _fma(a[1], b[1], a[0] * b[0]))


def camera_rays(K1: np.ndarray, w: int, h: int) -> np.ndarray:
    """Nc [3, h*w] (sl_system.py:353-365): ((u-cx)/fx, (v-cy)/fy, 1) / norm, the
    norm an add.reduce over the last axis: ((x*x + y*y) + 1*1)."""
    u, v = np.meshgrid(np.arange(w), np.arange(h))
    fx, fy, cx, cy = K1[0, 0], K1[1, 1], K1[0, 2], K1[1, 2]
    x = (u - cx) / fx
    y = (v - cy) / fy
    n = np.sqrt((x * x + y * y) + 1.0)
    return np.stack([(x / n).ravel(), (y / n).ravel(), (1.0 / n).ravel()])


def projector_planes(K2: np.ndarray, R: np.ndarray, T: np.ndarray, Wp: int, Hp: int):
    """(wPlaneCol [4, Wp], wPlaneRow [4, Hp]) as calibrate_final saves them
    (get_plane_from_proj_line, sl_system.py:367-403)."""
    fxp, fyp, cxp, cyp = float(K2[0, 0]), float(K2[1, 1]), float(K2[0, 2]), float(K2[1, 2])
    Ri = np.asarray(R, dtype=np.float64).T
    Tf = np.asarray(T, dtype=np.float64).reshape(3)
    C = [_dot3([-Ri[i, 0], -Ri[i, 1], -Ri[i, 2]], Tf) for i in range(3)]  # -R_inv @ T (:377)

    def plane(p1, p2):
        r1 = [_dot3(Ri[i], p1) for i in range(3)]
        r2 = [_dot3(Ri[i], p2) for i in range(3)]
        n = [r1[1] * r2[2] - r1[2] * r2[1],  # np.cross
             r1[2] * r2[0] - r1[0] * r2[2],
             r1[0] * r2[1] - r1[1] * r2[0]]
        nn = float(np.sqrt(_dot3(n, n)))
        n = [n[0] / nn, n[1] / nn, n[2] / nn]
        return [n[0], n[1], n[2], -_dot3(n, C)]

    col = np.empty((4, Wp))
    for c in range(Wp):  # is_col: pixels (c, 0) and (c, Hp) (:382-384, :397-398)
        x = (c - cxp) / fxp
        col[:, c] = plane([x, (0 - cyp) / fyp, 1.0], [x, (Hp - cyp) / fyp, 1.0])
    row = np.empty((4, Hp))
    for r in range(Hp):  # rows: pixels (0, r) and (Wp, r) (:386-387, :401-402)
        y = (r - cyp) / fyp
        row[:, r] = plane([(0 - cxp) / fxp, y, 1.0], [(Wp - cxp) / fxp, y, 1.0])
    return col, row


def calibration_products(K1, K2, R, T, w: int, h: int, Wp: int = 1920, Hp: int = 1080) -> dict:
    """The dict calibrate_final saves with scipy.io.savemat (:405-414)."""
    col, row = projector_planes(K2, R, T, Wp, Hp)
    return {"Nc": camera_rays(np.asarray(K1, dtype=np.float64), w, h), "Oc": np.zeros((3, 1)),
            "wPlaneCol": col, "wPlaneRow": row, "cam_K": np.asarray(K1), "proj_K": np.asarray(K2),
            "R": np.asarray(R), "T": np.asarray(T)}
