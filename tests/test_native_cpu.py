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


def _gitem(N, **kw):
    e = N.GemmItem()
    e.a = e.b = e.c = 0x7F0000000000
    e.m, e.n, e.lda, e.ldb, e.ldc = 256, 128, 256, 128, 128
    e.flags, e.f16, e.split, e.k_chunk = N.EPI_ACCUM, 0, 1, 0
    for k, v in kw.items():
        setattr(e, k, v)
    return e


@pytest.mark.parametrize("kw,msg", [(dict(m=100), b"m=100"), (dict(flags=64 | 512), b"flags"),
                                    (dict(split=3, k_chunk=320, flags=16), b"k_chunk 320"),
                                    (dict(split=3, k_chunk=384), b"OUT_F32"), (dict(lda=128), b"lda=128"),
                                    (dict(f16=2), b"f16=2"), (dict(a=0x7F0000000008), b"aligned")])
def test_grouped_gemm_rejects_bad_items_without_launching(kw, msg):
    """lrce_gemm_grouped validates every entry before any launch: shape multiples, epilogue flags (a
    bias gradient needs a bias), K slices (split x k_chunk must cover K exactly, slabs are stored),
    leading dims, operand format and alignment."""
    from lrce import _native as N
    items = (N.GemmItem * 2)(_gitem(N), _gitem(N, **kw))
    assert N.lib().lrce_gemm_grouped(items, 2, 1000, 1.0, None) == 1
    assert msg in N.lib().lrce_last_error(), N.lib().lrce_last_error()


@pytest.mark.skipif(torch.cuda.is_available(), reason="would launch on the GPU with fake pointers")
def test_grouped_gemm_host_path_returns_without_a_device():
    """100 valid entries of 9 shapes (more than one launch's 80-entry / 8-shape tables, bf16 and fp16,
    split and unsplit): the host side packs every launch and returns the HIP error as a status code."""
    from lrce import _native as N
    its = []
    for i in range(100):
        m = 128 * (1 + i % 9)
        its.append(_gitem(N, m=m, lda=m, f16=i % 2, split=1 + (i % 3 == 0) * 2, k_chunk=384 if i % 3 == 0 else 0,
                          flags=N.EPI_OUT_F32 if i % 3 == 0 else N.EPI_ACCUM, c=0x7F0000000000 + 0x100000 * i))
    items = (N.GemmItem * 100)(*its)
    assert N.lib().lrce_gemm_grouped(items, 100, 1000, 1.0, None, None) != 0
    s = (N.SlabSum * 1)()
    s[0].slabs, s[0].dst, s[0].n, s[0].split, s[0].accumulate = 0x7F0000000000, 0x7F0000100000, 6, 2, 1
    assert N.lib().lrce_slab_sum_grouped(s, 1, None) == 1 and b"n % 4" in N.lib().lrce_last_error()


def test_grouped_weight_gradient_packing(monkeypatch):
    """kernels.linear_dw_grouped's host packing (CPU tensors, the launch intercepted): per-entry shape /
    leading dims / flags / device alpha, and with K slices every weight and bias slab carved from one
    workspace, k_chunk a multiple of 64 covering T, the slab sums storing fresh weights and adding biases."""
    from lrce import kernels as K, _native as N
    calls = {}

    def fake_call(name, *args):
        calls[name] = args
    monkeypatch.setattr(K, "call", fake_call)
    monkeypatch.setattr(K, "stream_of", lambda t: None)
    T = 1000
    shapes = [(256, 384), (128, 256), (384, 128)]
    items = []
    for j, (O, I) in enumerate(shapes):
        dy = torch.zeros(T, O, dtype=torch.bfloat16)
        x = torch.zeros(T, 2 * I, dtype=torch.bfloat16)[:, :I]          # a column block: ldb = 2I
        dw, db = torch.zeros(O, I), (torch.zeros(O) if j != 1 else None)
        items.append((dy, x, dw, db, j == 0))
    K.linear_dw_grouped(items)
    arr = calls["lrce_gemm_grouped"][0]
    assert calls["lrce_gemm_grouped"][1:5] == (3, T, 1.0, None) and "lrce_slab_sum_grouped" not in calls
    for e, (dy, x, dw, db, store) in zip(arr, items):
        assert (e.m, e.n, e.lda, e.ldb, e.ldc, e.split) == (dw.shape[0], dw.shape[1], dw.shape[0], 2 * dw.shape[1],
                                                          dw.shape[1], 1)
        assert e.c == dw.data_ptr() and (e.bias or 0) == (db.data_ptr() if db is not None else 0)
        assert e.flags == ((N.EPI_OUT_F32 if store else N.EPI_ACCUM) | (N.EPI_BIAS_GRAD if db is not None else 0))
    calls.clear()
    K.linear_dw_grouped(items, split=3)
    arr = calls["lrce_gemm_grouped"][0]
    sums, nsum = calls["lrce_slab_sum_grouped"][0], calls["lrce_slab_sum_grouped"][1]
    kc = arr[0].k_chunk
    assert kc % 64 == 0 and (arr[0].split - 1) * kc < T <= arr[0].split * kc
    assert nsum == 5   # three weights + two biases
    k = 0
    for e, (dy, x, dw, db, store) in zip(arr, items):
        assert e.flags & N.EPI_OUT_F32 and e.split == arr[0].split
        assert sums[k].slabs == e.c and sums[k].dst == dw.data_ptr() and sums[k].n == dw.numel()
        assert sums[k].accumulate == int(not store)
        k += 1
        if db is not None:
            assert sums[k].slabs == e.bias and sums[k].dst == db.data_ptr() and sums[k].accumulate == 1
            k += 1
