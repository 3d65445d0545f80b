"""Calibration products: the tail of ``SLSystem.calibrate_final``
(server/sl_system.py:329-415), SURVEY.md §8(f)-4.

The reference calibrates the camera and projector with OpenCV
(``cv2.calibrateCamera`` / ``cv2.stereoCalibrate``, :331-345 -- checkerboard
detection and calibration are out of scope here, and cv2 is not in this
image), then derives what every later scan reads from ``calib.mat``: the
per-pixel camera rays ``Nc``, ``Oc`` and the projector column / row planes.
This module computes those products on the GPU (csrc/slcalib.hip, bit-identical
to the reference's NumPy/OpenBLAS evaluation) from the stereo parameters and
writes the same ``.mat`` file.
"""
from __future__ import annotations

import numpy as np
import scipy.io

from . import core

SCREEN_WIDTH = 1920   # config.py:16 (the projector the planes are built for)
SCREEN_HEIGHT = 1080  # config.py:18


def calibration_products(cam_K, proj_K, R, T, shape, screen=(SCREEN_WIDTH, SCREEN_HEIGHT), device=None,
                         rays: bool = True) -> dict:
    """The dict calibrate_final saves (sl_system.py:405-414): ``Nc`` [3, h*w],
    ``Oc`` zeros [3, 1], ``wPlaneCol`` [4, Wp], ``wPlaneRow`` [4, Hp], ``cam_K``,
    ``proj_K``, ``R``, ``T``.  ``shape`` is the camera image size as OpenCV
    gives it, ``(w, h)`` (:350).  ``rays=False`` skips ``Nc`` (3x1 zeros
    instead: the reconstruction then regenerates pinhole rays from ``cam_K``,
    sl_system.py:607-621 -- 24 B/px less to store)."""
    w, h = (int(shape[0]), int(shape[1]))
    wp, hp = (int(screen[0]), int(screen[1]))
    eng = core.engine(device)
    nc, col, row = eng.calib_products(cam_K, proj_K, R, T, w, h, wp, hp, rays=rays)
    eng.sync()
    return {"Nc": nc.cpu().numpy() if nc is not None else np.zeros((3, 1)), "Oc": np.zeros((3, 1)),
            "wPlaneCol": col.cpu().numpy(), "wPlaneRow": row.cpu().numpy(),
            "cam_K": np.asarray(cam_K, dtype=np.float64), "proj_K": np.asarray(proj_K, dtype=np.float64),
            "R": np.asarray(R, dtype=np.float64), "T": np.asarray(T, dtype=np.float64)}


def save_calibration(output_file: str, products: dict) -> None:
    """scipy.io.savemat, as calibrate_final writes calib.mat (:405-414)."""
    scipy.io.savemat(output_file, products)


def calibrate_final_from_stereo(cam_K, proj_K, R, T, shape, output_file: str,
                                screen=(SCREEN_WIDTH, SCREEN_HEIGHT), device=None) -> dict:
    """calibrate_final after its stereo calibration: products -> ``output_file``."""
    prod = calibration_products(cam_K, proj_K, R, T, shape, screen, device)
    save_calibration(output_file, prod)
    return prod
