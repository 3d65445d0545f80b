"""Calibration-products oracle (oracle/calib_oracle.py) vs the reference's own
calibrate_final output (tests/golden/calib_*.npz, made by
tests/golden/make_calib_golden.py), bit for bit.  CPU only."""
import glob
import json
import os

import numpy as np
import pytest

from oracle import calib_oracle as co

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "calib_*.npz")))


def load(path):
    z = np.load(path)
    return json.loads(str(z["meta"])), z


def test_fixtures_present():
    assert len(GOLD) >= 2


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_oracle_matches_reference_calibrate_final(path):
    meta, z = load(path)
    prod = co.calibration_products(z["in_K1"], z["in_K2"], z["in_R"], z["in_T"], meta["w"], meta["h"],
                                   meta["screen_w"], meta["screen_h"])
    for k in ("Nc", "Oc", "wPlaneCol", "wPlaneRow"):
        assert prod[k].shape == z[k].shape, k
        np.testing.assert_array_equal(prod[k], z[k], err_msg=k)
    for k, src in (("cam_K", "in_K1"), ("proj_K", "in_K2"), ("R", "in_R"), ("T", "in_T")):
        np.testing.assert_array_equal(z[k], z[src])


def test_planes_are_unit_and_contain_projector_centre():
    _, z = load(GOLD[0])
    col = z["wPlaneCol"]
    np.testing.assert_allclose(np.linalg.norm(col[:3], axis=0), 1.0, atol=1e-15)
    C = (-z["in_R"].T @ z["in_T"]).ravel()
    np.testing.assert_allclose(col[:3].T @ C + col[3], 0.0, atol=1e-9)
