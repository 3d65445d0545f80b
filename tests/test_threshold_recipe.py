"""The adaptive-mask threshold recipe k_stats implements, modelled in Python.

k_stats never sorts: it builds a 256-bin histogram of the black plane and
max(white - black), then evaluates numpy 2.x's float32 percentile
(method='linear') from the histogram's order statistics and turns the float32
thresholds into integer ones (white and contrast are integers, so x > t <=>
x > floor(t)).  This test pins that recipe against np.percentile / the oracle
mask on many random and adversarial inputs; tests/test_gpu_parity.py checks
the kernel against the same references.
"""
import numpy as np
import pytest

from oracle import sl_oracle as o


def recipe(white, black):
    n = black.size
    hist = np.bincount(black.ravel(), minlength=256)
    cdf = np.cumsum(hist)
    q = np.float32(95) / np.float32(100)
    fn1 = np.float32(n - 1)
    vi = np.float32(fn1 * q)
    if vi >= fn1:
        kp = kn = n - 1
        gamma = np.float32(0)
    else:
        pf = np.float32(np.floor(vi))
        kp, kn = int(pf), int(np.float32(pf + np.float32(1)))
        gamma = np.float32(vi - pf)
    a = np.float32(np.searchsorted(cdf, kp, side="right"))
    b = np.float32(np.searchsorted(cdf, kn, side="right"))
    diff = np.float32(b - a)
    nf = np.float32(a + np.float32(diff * gamma))
    if gamma >= np.float32(0.5):
        nf = np.float32(b - np.float32(diff * np.float32(np.float32(1) - gamma)))
    dr = np.float32(int((white.astype(np.int32) - black.astype(np.int32)).max()))
    tw = int(np.floor(np.float32(nf * np.float32(1.5))))
    tc = int(np.floor(np.float32(dr * np.float32(0.05))))
    return nf, dr, tw, tc


def _cases():
    rng = np.random.default_rng(42)
    for i in range(300):
        h, w = rng.integers(1, 90, 2)
        kind = i % 6
        if kind == 0:
            black = rng.integers(0, 256, (h, w))
        elif kind == 1:
            black = rng.integers(0, 16, (h, w))
        elif kind == 2:
            black = np.where(rng.random((h, w)) < 0.07, rng.integers(200, 256, (h, w)), rng.integers(0, 6, (h, w)))
        elif kind == 3:
            black = np.full((h, w), rng.integers(0, 256))
        elif kind == 4:
            black = rng.choice([0, 255], (h, w))
        else:
            black = np.clip(rng.normal(20, 8, (h, w)), 0, 255).astype(int)
        white = np.clip(black + rng.integers(-60, 230, (h, w)), 0, 255)
        yield white.astype(np.uint8), black.astype(np.uint8)
    # full-size frame shapes (virtual index handling at n ~ 8.3M and 12M)
    for h, w in ((2160, 3840), (3000, 4000), (720, 1280)):
        black = rng.integers(0, 40, (h, w)).astype(np.uint8)
        white = np.clip(black.astype(int) + 150, 0, 255).astype(np.uint8)
        yield white, black


def test_recipe_equals_numpy_percentile_and_oracle_mask():
    for white, black in _cases():
        nf, dr, tw, tc = recipe(white, black)
        nf_ref, dr_ref = o.adaptive_thresholds(white, black)
        assert np.float32(nf).view(np.uint32) == np.float32(nf_ref).view(np.uint32), (white.shape, nf, nf_ref)
        assert dr == dr_ref
        mask = (white.astype(int) > tw) & ((white.astype(int) - black.astype(int)) > tc)
        np.testing.assert_array_equal(mask, o.valid_mask(white, black))
