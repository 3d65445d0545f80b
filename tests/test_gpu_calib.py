"""Calibration products on the GPU (csrc/slcalib.hip through sl_calib_products)
vs the reference's calibrate_final output (tests/golden/calib_*.npz) and the
oracle, bit for bit (GPU only)."""
import glob
import json
import os

import numpy as np
import pytest
import torch

from oracle import calib_oracle as co

pytestmark = pytest.mark.gpu

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "calib_*.npz")))


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_gpu_calib_products_match_reference(path, tmp_path):
    from structured_light_for_3d_model_replication_amd import calibration
    z = np.load(path)
    meta = json.loads(str(z["meta"]))
    out = tmp_path / "calib.mat"
    prod = calibration.calibrate_final_from_stereo(z["in_K1"], z["in_K2"], z["in_R"], z["in_T"],
                                                   (meta["w"], meta["h"]), str(out),
                                                   screen=(meta["screen_w"], meta["screen_h"]))
    for k in ("Nc", "Oc", "wPlaneCol", "wPlaneRow"):
        np.testing.assert_array_equal(prod[k], z[k], err_msg=k)
    import scipy.io
    m = scipy.io.loadmat(str(out))
    for k in ("Nc", "Oc", "wPlaneCol", "wPlaneRow", "cam_K", "proj_K", "R", "T"):
        np.testing.assert_array_equal(m[k], z[k], err_msg=k)


def test_gpu_calib_4k_rays_and_wide_projector_vs_oracle():
    """Full 4K camera (8.3M rays) and a 1024x768 projector vs the oracle; the
    4K rays also equal the pinhole rays the reconstruction kernels derive
    from cam_K (sl_set_calib drops such an Nc)."""
    from structured_light_for_3d_model_replication_amd import core, synth
    rig = synth.Rig(H=2160, W=3840, Wp=1024, Hp=768)
    eng = core.engine(0)
    nc, col, row = eng.calib_products(rig.cam_K, rig.proj_K, rig.R, rig.T, rig.W, rig.H, rig.Wp, rig.Hp)
    eng.sync()
    np.testing.assert_array_equal(nc.cpu().numpy(), co.camera_rays(rig.cam_K, rig.W, rig.H))
    ocol, orow = co.projector_planes(rig.proj_K, rig.R, rig.T, rig.Wp, rig.Hp)
    np.testing.assert_array_equal(col.cpu().numpy(), ocol)
    np.testing.assert_array_equal(row.cpu().numpy(), orow)
    cal = synth.make_calibration(rig, with_Nc=True)
    np.testing.assert_array_equal(nc.cpu().numpy(), cal["Nc"])


def test_gpu_calib_errors():
    from structured_light_for_3d_model_replication_amd import core
    eng = core.engine(0)
    with pytest.raises(ValueError):
        eng.calib_products(np.eye(3), np.eye(3), np.eye(3), np.zeros(3), 0, 10)
    with pytest.raises(ValueError):
        eng.calib_products(np.eye(3), np.eye(3), np.eye(3), np.zeros(4), 10, 10)
