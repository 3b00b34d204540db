"""C ABI checks that need no GPU: the library loads, exports every symbol include/oflow.h declares, and its
argument validation / helpers behave (no kernel is launched here)."""
import ctypes
import os
import re

import pytest

from conftest import REPO
from optical_flow import _native


def _declared_symbols():
    text = open(os.path.join(REPO, "include", "oflow.h")).read()
    return sorted(set(re.findall(r"^\s*(?:[\w*]+\s+)+\**(oflow_\w+)\s*\(", text, flags=re.M)))


def test_header_and_binding_agree():
    assert _declared_symbols() == sorted(_native.SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_native.library_path())
    for name in _declared_symbols():
        assert hasattr(lib, name), name


def test_abi_version_and_status_strings():
    lib = _native.load()
    assert lib.oflow_abi_version() == _native.ABI_VERSION
    assert lib.oflow_status_string(0) == b"ok"
    assert b"2 pixels" in lib.oflow_status_string(_native.E_TINY)
    for code in range(-7, 0):
        assert lib.oflow_status_string(code) != b"unknown oflow status"


def test_pyramid_dims_floor_halving():
    # corr.py:53 avg_pool2d(2, stride=2): floor; Sintel 55x128 -> 27x64 -> 13x32 -> 6x16
    assert _native.pyramid_dims(55, 128, 4) == [(55, 128), (27, 64), (13, 32), (6, 16)]
    assert _native.pyramid_dims(47, 156, 4) == [(47, 156), (23, 78), (11, 39), (5, 19)]
    assert _native.pyramid_dims(135, 240, 4) == [(135, 240), (67, 120), (33, 60), (16, 30)]
    with pytest.raises(RuntimeError):
        _native.pyramid_dims(10, 10, 9)


def test_argument_errors_are_reported_without_launch():
    lib = _native.load()
    ptrs = (ctypes.c_void_p * 4)()
    assert lib.oflow_corr_pyramid_f32(None, None, 1, 256, 16, 16, 4, ptrs, None) == -1
    hs = (ctypes.c_int * 4)(16, 8, 4, 1)
    ws = (ctypes.c_int * 4)(16, 8, 4, 2)
    fake = (ctypes.c_void_p * 4)(4096, 4096, 4096, 4096)
    # level 3 is 1 px high: the reference would divide by H_l - 1 = 0 (Q3) -> OFLOW_E_TINY
    assert lib.oflow_corr_lookup_f32(fake, hs, ws, 4, 4096, 1, 16, 16, 4, 4096, None) == _native.E_TINY
    assert lib.oflow_corr_lookup_f32(fake, hs, ws, 4, 4096, 1, 16, 16, 9, 4096, None) == -5
    assert lib.oflow_grid_warp_f32(4096, 4096, 1, 3, 4, 4, 7, 0, 0, 4096, None) == -6
    assert lib.oflow_grid_warp_f32(4096, 4096, 1, 3, 4, 4, 0, 5, 0, 4096, None) == -6
