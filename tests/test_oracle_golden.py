"""The CPU oracle against every golden fixture produced by the reference itself."""
import numpy as np
import pytest

from oracle import sl_oracle as o
from tests import golden_io as g

STACK_CASES = g.names(func={"sl", "mp", "generate_cloud"})


@pytest.mark.parametrize("name", STACK_CASES)
def test_decode_and_cloud_bit_exact(name):
    d = g.load(name)
    m = d["meta"]
    col, row, mask, P, C = o.decode_triangulate(list(d["stack"]), d["texture"], d["calib"],
                                               m["n_cols"], m["n_rows"], m["mask_mode"])
    assert col.dtype == np.int32 and row.dtype == np.int32 and mask.dtype == bool
    np.testing.assert_array_equal(col, d["col_map"])
    np.testing.assert_array_equal(row, d["row_map"])
    np.testing.assert_array_equal(mask, d["mask"])
    assert P.dtype == np.float64 and C.dtype == np.uint8
    # bitwise: same f64 bits, same colours, same order
    assert P.shape == d["P"].shape
    np.testing.assert_array_equal(P.view(np.uint64), d["P"].view(np.uint64))
    np.testing.assert_array_equal(C, d["C"])


def test_reconstruct_only_colour_clip():
    d = g.load("sl_reconstruct_colour_clip")
    P, C = o.reconstruct_point_cloud(d["col_map"], d["row_map"], d["mask"], d["texture"], d["calib"])
    np.testing.assert_array_equal(P.view(np.uint64), d["P"].view(np.uint64))
    np.testing.assert_array_equal(C, d["C"])


@pytest.mark.parametrize("name", ["sl_generate_cloud_e2e", "mp_fixed_mask"])
def test_ply_bytes(name):
    d = g.load(name)
    assert o.ply_text(d["P"], d["C"]) == g.ply_text(d["meta"]["ply"])


def test_adaptive_threshold_pins():
    d = g.load("adaptive_threshold_pins")
    for k in range(d["meta"]["n"]):
        w, b = d[f"white_{k}"], d[f"black_{k}"]
        np.testing.assert_array_equal(o.valid_mask(w, b), d[f"mask_{k}"])
        nf, _ = o.adaptive_thresholds(w, b)
        assert np.float32(nf).view(np.uint32) == d[f"nf_{k}"].view(np.uint32)


def test_error_behaviour():
    d = g.load("errors")
    errs = d["meta"]["errors"]
    n_img = {"three": 3, "odd9": 9, "odd15": 15}
    for tag, exc_name in errs.items():
        imgs = list(d["stack"][: n_img[tag]])
        if exc_name == "ok":
            o.gray_decode_images(imgs, 16, 8)
            continue
        with pytest.raises({"ValueError": ValueError, "IndexError": IndexError}[exc_name]):
            o.gray_decode_images(imgs, 16, 8)
