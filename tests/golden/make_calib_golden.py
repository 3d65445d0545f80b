"""Golden fixtures for the calibration products, made by
running the REFERENCE's own ``SLSystem.calibrate_final`` (server/sl_system.py:329-415)
in the build container (it reads /root/reference):

    python tests/golden/make_calib_golden.py

``calibrate_final`` calibrates with OpenCV (absent here) and then derives the
products the scanner uses: the per-pixel camera rays ``Nc``, ``Oc`` and the
projector column / row planes ``wPlaneCol`` / ``wPlaneRow``, written with
``scipy.io.savemat``.  The method is taken from the source with ``ast`` and
compiled unmodified; its OpenCV calls are stubbed to RETURN given stereo
parameters (K1, K2, R, T) -- the stubs compute nothing -- and
``messagebox.showinfo`` is a no-op.  All arithmetic executed after the stubs is
the reference's (NumPy 2.2.6 + this image's OpenBLAS 0.3.29, whose 3-term
dot / matmul kernels are left-to-right FMA chains; see oracle/calib_oracle.py).

Only inputs and the .mat outputs (as arrays) are stored, in calib_*.npz.
"""
from __future__ import annotations

import ast
import json
import math
import os
import sys
import tempfile
import types

import numpy as np
import scipy.io

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _screen():
    tree = ast.parse(open(os.path.join(REF, "server", "config.py"), encoding="utf-8").read())
    vals = {}
    for n in tree.body:
        if isinstance(n, ast.Assign) and isinstance(n.targets[0], ast.Name) and \
                n.targets[0].id in ("SCREEN_WIDTH", "SCREEN_HEIGHT"):
            vals[n.targets[0].id] = ast.literal_eval(n.value)
    return vals["SCREEN_WIDTH"], vals["SCREEN_HEIGHT"]


def load_calibrate_final(stereo):
    p = os.path.join(REF, "server", "sl_system.py")
    tree = ast.parse(open(p, encoding="utf-8").read())
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "SLSystem")
    fn = next(n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == "calibrate_final")
    sw, sh = _screen()
    K1, K2, R, T = stereo["K1"], stereo["K2"], stereo["R"], stereo["T"]
    cv2 = types.SimpleNamespace(
        calibrateCamera=lambda obj, img, size, a, b: (0.0, K1 if size == stereo["shape"] else K2,
                                                      np.zeros(5), None, None),
        stereoCalibrate=lambda *a, **k: (0.25, K1, np.zeros(5), K2, np.zeros(5), R, T, None, None),
        CALIB_FIX_INTRINSIC=256)
    ns = {"np": np, "scipy": scipy, "cv2": cv2, "SCREEN_WIDTH": sw, "SCREEN_HEIGHT": sh,
          "messagebox": types.SimpleNamespace(showinfo=lambda *a, **k: None), "__name__": "ref"}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), p, "exec"), ns)
    return ns["calibrate_final"], (sw, sh)


def rot(axis, deg):
    a = np.asarray(axis, dtype=np.float64)
    a = a / np.linalg.norm(a)
    t = math.radians(deg)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + math.sin(t) * K + (1 - math.cos(t)) * (K @ K)


def run_case(name, w, h, K1, K2, R, T):
    stereo = {"K1": K1, "K2": K2, "R": R, "T": T, "shape": (w, h)}
    fn, (sw, sh) = load_calibrate_final(stereo)
    me = types.SimpleNamespace(load_calib_data=lambda base, poses: ([], [], [], (w, h), None))
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "calib.mat")
        fn(me, tmp, [], out)
        m = scipy.io.loadmat(out)
    arrays = {k: np.asarray(m[k]) for k in ("Nc", "Oc", "wPlaneCol", "wPlaneRow", "cam_K", "proj_K", "R", "T")}
    meta = {"w": w, "h": h, "screen_w": sw, "screen_h": sh, "func": "calibrate_final",
            "ref": "server/sl_system.py:329-415"}
    np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta),
                        in_K1=K1, in_K2=K2, in_R=R, in_T=T, **arrays)
    print(name, {k: v.shape for k, v in arrays.items()})


def main():
    # the SURVEY §8(d) rig at a small camera: fx = fy = 0.9 W, centred; projector
    # 1920x1080 rotated 15 deg about y, 200 mm baseline
    w, h = 64, 40
    K1 = np.array([[0.9 * w, 0, (w - 1) / 2], [0, 0.9 * w, (h - 1) / 2], [0, 0, 1.0]])
    K2 = np.array([[1.1 * 1920, 0, 959.5], [0, 1.1 * 1920, 539.5], [0, 0, 1.0]])
    run_case("calib_rig_64x40", w, h, K1, K2, rot((0, 1, 0), 15.0), np.array([[-200.0], [0.0], [0.0]]))
    # a general stereo pair: off-centre principal points, fx != fy, tilted rotation axis
    w, h = 45, 31
    K1 = np.array([[51.37, 0, 21.83], [0, 49.91, 16.07], [0, 0, 1.0]])
    K2 = np.array([[2087.3, 0, 941.2], [0, 2101.9, 563.8], [0, 0, 1.0]])
    run_case("calib_general_45x31", w, h, K1, K2, rot((0.3, 0.9, -0.2), 11.7),
             np.array([[-187.25], [13.5], [-21.125]]))


if __name__ == "__main__":
    sys.exit(main())
