"""The C ABI library: builds, loads and exports exactly what include/slgpu.h declares."""
import os
import re

import pytest

from structured_light_for_3d_model_replication_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    text = open(os.path.join(REPO, "include", "slgpu.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(sl_[a-z_]+)\s*\(", text))


def test_header_matches_binding_table():
    assert _declared() == set(_lib.EXPORTS)


def test_library_loads_and_exports_every_symbol():
    lib = _lib.load()
    for name in _lib.EXPORTS:
        assert getattr(lib, name) is not None
    assert lib.sl_abi_version() == 1


def test_error_mapping():
    with pytest.raises(ValueError):
        _lib.check(_lib.SL_EINVAL, None, "x")
    with pytest.raises(IndexError):
        _lib.check(_lib.SL_EINDEX, None, "x")
    with pytest.raises(_lib.SLError):
        _lib.check(_lib.SL_EHIP, None, "x")
    _lib.check(_lib.SL_OK)


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from structured_light_for_3d_model_replication_amd import core
    with pytest.raises(RuntimeError):
        core.Reconstructor()
    with pytest.raises(RuntimeError):
        core.engine()
