"""CPU-side checks of the C-ABI library: it loads, exports every entry point include/lrce_hip.h
declares, and rejects bad arguments with an error message (no compute calls without a GPU)."""
import ctypes
import os
import re

import pytest
import torch

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


@pytest.mark.skipif(torch.cuda.is_available(), reason="would launch on the GPU with fake pointers")
@pytest.mark.parametrize("f16,a_km,b_km", [(0, 1, 1), (1, 1, 1), (1, 1, 0), (1, 0, 0), (0, 0, 0)])
def test_gemm_dispatch_returns_without_a_device(f16, a_km, b_km):
    """Every LDS-DMA dispatch branch (bf16 / fp16, the forward, dX and dW layouts) runs its host path to
    the launch and returns the HIP error as a status code when no device is visible (a host-side fault in
    the launcher — e.g. a dispatch lambda that falls off its end — would crash this process)."""
    from lrce import _native
    d = _native.GemmDesc()
    d.a = d.b = d.c = 0x7F0000000000
    d.m, d.n, d.k, d.batch = 320, 768, 768, 1
    d.lda = d.ldb = d.ldc = 768
    d.a_kmajor, d.b_kmajor, d.f16, d.alpha = a_km, b_km, f16, 1.0
    rc = _native.lib().lrce_gemm(ctypes.byref(d), None)
    assert rc != 0


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


def test_bias_gradient_bins_map_to_relative_position_index():
    """The window backward bins (query i, key j) by code(i) - code(j) + off; wattn_bin_rows maps every
    bin to the relative_position_index row all its pairs share (video_swin_ori.py:133-148): every row
    the index uses is hit by exactly one bin, and each bin's pairs agree with the index."""
    import torch
    from lrce import kernels as K
    from lrce.feature_extractor.video_swin import relative_position_index
    index = relative_position_index((8, 7, 7))
    for win in ((3, 7, 7), (2, 7, 7), (8, 7, 7)):
        wd, wh, ww = win
        n = wd * wh * ww
        rows = K.wattn_bin_rows(index, win)
        assert rows.dtype == torch.int32 and rows.numel() == K.wattn_n_bins(win)
        used = index[:n, :n].unique()
        assert torch.equal(rows[rows >= 0].long().sort().values, used)
        x = torch.arange(n)
        code = ((x // (wh * ww)) * (2 * wh - 1) + (x // ww) % wh) * (2 * ww - 1) + x % ww
        off = ((wd - 1) * (2 * wh - 1) + (wh - 1)) * (2 * ww - 1) + (ww - 1)
        b = code[:, None] - code[None, :] + off
        assert torch.equal(rows.long()[b], index[:n, :n])
    bad = index.clone()
    bad[0, 1], bad[1, 2] = bad[1, 2], bad[0, 1] + 1
    with pytest.raises(ValueError):
        K.wattn_bin_rows(bad, (3, 7, 7))


def test_torch_library_ops_registered_with_fake_shapes():
    """lrce/ops.py registers torch.ops.lrce.* with schemas and fake (shape-only) implementations;
    shape propagation runs on meta tensors without a GPU (no compute)."""
    from lrce import ops
    for name in ops.registered():
        assert hasattr(torch.ops.lrce, name), name
    bf = torch.bfloat16
    y = torch.ops.lrce.linear(torch.empty(4, 8, device="meta", dtype=bf), torch.empty(6, 8, device="meta", dtype=bf),
                              None, False, True)
    assert y.shape == (4, 6) and y.dtype == torch.float32
    dx = torch.ops.lrce.linear_dx(torch.empty(4, 6, device="meta", dtype=bf), torch.empty(6, 8, device="meta", dtype=bf))
    assert dx.shape == (4, 8)
    out, qkv, lse = torch.ops.lrce.window_attention(
        torch.empty(2 * 147, 256, device="meta", dtype=bf), torch.empty(768, 256, device="meta", dtype=bf),
        torch.empty(768, device="meta"), torch.empty(2535, 8, device="meta"),
        torch.empty(392, 392, device="meta", dtype=torch.int64), 2, 8)
    assert out.shape == (294, 256) and qkv.shape == (294, 768) and lse.shape == (2, 8, 160)


def test_stale_library_is_refused_whole(monkeypatch):
    """A shared library missing one declared entry point (a stale build) is refused on EVERY call:
    never handed out half-declared (undeclared ctypes entries would pass 64-bit pointers as ints)."""
    import ctypes
    from lrce import _native as N
    monkeypatch.setattr(N, "_lib", None)
    monkeypatch.setitem(N._SIGS, "lrce_no_such_entry_point", [])
    for _ in range(2):
        with pytest.raises(N.NativeError, match="stale build"):
            N.lib()
    assert N._lib is None
