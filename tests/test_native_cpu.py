"""CPU-side checks of the C-ABI library: it loads, exports every entry point include/lrce_hip.h
declares, and rejects bad arguments with an error message (no compute calls without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import REPO


def _header_symbols():
    src = open(os.path.join(REPO, "include", "lrce_hip.h")).read()
    return sorted(set(re.findall(r"\b(lrce_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from lrce import _native
    lib = _native.lib()
    missing = [s for s in _header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(_header_symbols()) == set(_native.exported_symbols())
    assert lib.lrce_version() == 1


def test_gemm_rejects_bad_shapes_without_launching():
    from lrce import _native
    d = _native.GemmDesc()
    d.a = d.b = d.c = 0x1000
    d.m, d.n, d.k, d.batch = 16, 16, 12, 1  # K % 8 != 0 for K-major operands
    d.a_kmajor = d.b_kmajor = 1
    d.lda = d.ldb = 16
    rc = _native.lib().lrce_gemm(ctypes.byref(d), None)
    assert rc == 1
    assert b"% 8" in _native.lib().lrce_last_error()


def test_wattn_rejects_unsupported_window():
    from lrce import _native
    rc = _native.lib().lrce_wattn_fwd(0x1000, 0x1000, None, 0x1000, 0x1000, 4, 100, 4, None)
    assert rc == 1
    assert b"outside" in _native.lib().lrce_last_error()


def test_kernels_refuse_cpu_tensors():
    import torch
    from lrce import kernels, _native
    x = torch.zeros(8, 8, dtype=torch.bfloat16)
    with pytest.raises(_native.NativeError):
        kernels.linear(x, x)
