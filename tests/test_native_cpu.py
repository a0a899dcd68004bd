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
    rc = _native.lib().lrce_wattn_fwd_grouped(0x1000, 0x1000, None, None, 1, 0x1000, 0x1000, 4, 100, 4, None)
    assert rc == 1
    assert b"outside" in _native.lib().lrce_last_error()


def test_kernels_refuse_cpu_tensors():
    import torch
    from lrce import kernels, _native
    x = torch.zeros(8, 8, dtype=torch.bfloat16)
    with pytest.raises(_native.NativeError):
        kernels.linear(x, x)


def test_dbias_csr_inverts_relative_position_index():
    """The bias-gradient CSR (host-built) lists every valid (query, key) pair of the padded 160x160
    per-lane tile layout exactly once, under its relative_position_index row, ascending per row."""
    import torch
    from lrce import kernels as K
    from lrce.feature_extractor.video_swin import relative_position_index
    n = 147
    index = relative_position_index((8, 7, 7))
    off, el, n_bins = K.wattn_dbias_csr(index, n, 2535)
    assert n_bins == 2535 and off.shape == (2536,) and int(off[-1]) == n * n == el.numel()
    assert el.unique().numel() == el.numel()
    reg, lane, tile = el & 15, (el >> 4) & 63, el // 1024
    qi = (tile // 5) * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
    kj = (tile % 5) * 32 + (lane & 31)
    assert int(qi.max()) < n and int(kj.max()) < n
    rows = torch.repeat_interleave(torch.arange(2535), (off[1:] - off[:-1]).long())
    assert torch.equal(index[qi.long(), kj.long()], rows)
    for b in range(0, 2535, 97):
        seg = el[off[b]:off[b + 1]]
        assert torch.equal(seg, seg.sort().values)
