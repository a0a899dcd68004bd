"""Tensor-level wrappers over the C ABI (lrce._native).  Every function here launches hand-written
gfx950 kernels from liblrce_hip.so on the current HIP stream; none computes with PyTorch.

Conventions: activations are 2-D row-major [rows, features]; weights are nn.Linear layout
[out, in]; "bf16" tensors are torch.bfloat16; gradients of parameters are f32 and accumulated.
"""
import ctypes
import math

import torch

from . import _native as N
from ._native import ptr, stream_of, call

BF16 = torch.bfloat16
F16 = torch.float16
F32 = torch.float32
NUM_CU = 256
_SPLIT_PER_CU = 2            # split-K blocks per CU
_SPLIT_MIN_DEPTH = 1024       # shallowest K slice


class KernelTimer:
    """Brackets selected launches with HIP events on the launch stream (bench.py roofline):
    `with KernelTimer("wattn_fwd") as kt: ...` then kt.mean_ms(), kt.calls, kt.flops."""
    active = None

    def __init__(self, *names, detail=False):
        self.names = set(names)
        self.events = {n: [] for n in names}
        self.flops = {n: 0.0 for n in names}
        self.bytes = {n: 0.0 for n in names}
        self.detail = {} if detail else None   # (name, key) -> [events], flops per launch

    def __enter__(self):
        KernelTimer.active = self
        return self

    def __exit__(self, *a):
        KernelTimer.active = None

    def wrap(self, name, stream_tensor, fn, flops=0.0, nbytes=0.0, key=None):
        if name not in self.names:
            return fn()
        s = torch.cuda.current_stream(stream_tensor.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r = fn()
        e1.record(s)
        self.events[name].append((e0, e1))
        if self.detail is not None:
            ent = self.detail.setdefault((name, key), [[], 0.0])
            ent[0].append((e0, e1))
            ent[1] += flops
        self.flops[name] += flops
        self.bytes[name] += nbytes
        return r

    def calls(self, name):
        return len(self.events[name])

    def total_ms(self, name):
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.events[name])

    def mean_ms(self, name):
        return self.total_ms(name) / max(1, self.calls(name))

    def summary(self, name):
        """(calls, mean ms per launch, algorithmic TFLOP/s, algorithmic GB/s) for one kernel family."""
        n, t = self.calls(name), self.total_ms(name)
        if n == 0 or t <= 0:
            return n, None, None, None
        return n, t / n, self.flops[name] / t / 1e9, self.bytes[name] / t / 1e6

    def breakdown(self):
        """[(name, key, calls, total ms, TFLOP/s)] per launch shape, largest total first (detail=True)."""
        torch.cuda.synchronize()
        rows = []
        for (name, key), (evs, fl) in (self.detail or {}).items():
            t = sum(a.elapsed_time(b) for a, b in evs)
            rows.append((name, key, len(evs), t, fl / max(t, 1e-9) / 1e9))
        return sorted(rows, key=lambda r: -r[3])


def _timed(name, stream_tensor, fn, flops=0.0, nbytes=0.0, key=None):
    kt = KernelTimer.active
    if kt is None:
        return fn()
    return kt.wrap(name, stream_tensor, fn, flops, nbytes, key)


def _ld(t):
    """Row pitch (elements) of a row-major matrix operand: a column block of a wider matrix has the
    wider matrix's pitch."""
    return t.stride(-2) if t.dim() >= 2 else t.shape[-1]


def _chk(t, dtype=None, name="tensor"):
    if t is None:
        return
    if not t.is_cuda:
        raise N.NativeError(f"{name} must be a HIP device tensor (no CPU fallback on the product path)")
    if dtype is not None and t.dtype != dtype:
        raise N.NativeError(f"{name}: expected {dtype}, got {t.dtype}")


def gemm(a, b, c, m, n, k, *, a_kmajor=True, b_kmajor=True, lda=None, ldb=None, ldc=None, flags=0, bias=None,
         aux=None, ld_aux=0, aux_out=None, ld_aux_out=0, a_map=None, c_map=None, alpha=1.0, split_k=1,
         scale_cols=0, scale_val=1.0, row_scale=None, rows_per_scale=1, a_row_scale=None, a_rows_per_scale=1,
         batch=1, stride_a=0, stride_b=0, stride_c=0, workspace=None, drop=None, f16=False, ln=None, alpha_dev=None,
         stride_bias=0, stride_alpha=0):
    """C (+)= epi(alpha * A(m,k) B(n,k)) — see include/lrce_hip.h LrceGemmDesc.  drop = (p, seed, group):
    nn.Dropout fused into the epilogue (exact-f32 skinny path; same mask as dropout()).  f16: every
    16-bit tensor (A, B, 16-bit C, aux_out) is torch.float16 (the BERT forward).  ln: a LayerNorm
    prologue on A (ln_fwd_prologue / ln_bwd_prologue -> lrce_gemm_ln).  alpha_dev: a device f32 read
    as alpha (the inverse gradient scale of grad_scale()); stride_alpha: its batch stride (floats)."""
    _chk(a, None, "A"); _chk(b, None, "B"); _chk(c, None, "C")
    a_f32 = a.dtype == F32
    b_f32 = b.dtype == F32
    b_half = a_f32 and b.dtype == F16 and not f16   # fp16 weights, f32 activations and arithmetic
    h = F16 if f16 else BF16
    if (not a_f32 and a.dtype != h) or (not b_f32 and not b_half and b.dtype != h):
        raise N.NativeError(f"gemm: operands must be {h} or f32")
    if lda is None:
        lda = k if a_kmajor else m
    if ldb is None:
        ldb = k if b_kmajor else n
    if ldc is None:
        ldc = n
    d = N.GemmDesc()
    d.a, d.b, d.c = ptr(a), ptr(b), ptr(c)
    d.lda, d.ldb, d.ldc = lda, ldb, ldc
    d.stride_a, d.stride_b, d.stride_c = stride_a, stride_b, stride_c
    d.stride_bias = stride_bias
    d.stride_alpha = stride_alpha
    d.m, d.n, d.k, d.batch = m, n, k, batch
    d.a_kmajor, d.b_kmajor, d.a_f32 = int(a_kmajor), int(b_kmajor), int(a_f32)
    d.flags, d.split_k = flags, split_k
    d.bias, d.aux, d.ld_aux = ptr(bias), ptr(aux), ld_aux
    d.aux_out, d.ld_aux_out = ptr(aux_out), ld_aux_out
    d.a_map, d.c_map = ptr(a_map), ptr(c_map)
    d.alpha, d.scale_cols, d.scale_val = alpha, scale_cols, scale_val
    d.row_scale, d.rows_per_scale = ptr(row_scale), rows_per_scale
    d.a_row_scale, d.a_rows_per_scale = ptr(a_row_scale), a_rows_per_scale
    d.b_f32 = 2 if b_half else int(b_f32)
    d.f16 = int(f16)
    if alpha_dev is not None:
        _chk(alpha_dev, F32, "alpha_dev")
        d.alpha_dev = ptr(alpha_dev)
    if workspace is not None:
        d.workspace, d.workspace_elems = ptr(workspace), workspace.numel()
    if drop is not None and drop[0] > 0:
        d.drop_p, d.drop_seed, d.drop_group = float(drop[0]), drop[1] & (2 ** 64 - 1), int(drop[2])
    if ln is not None:
        _timed("gemm_f32", c, lambda: call("lrce_gemm_ln", ctypes.byref(d), ctypes.byref(ln), stream_of(c)),
               flops=2.0 * m * n * k, key=(m, n, k, 1, "AK", "BK" if b_kmajor else "BN", f"ln{ln.mode}", 1, flags))
        return
    _timed("gemm_f32" if (b_f32 or b_half) else "gemm", c, lambda: call("lrce_gemm", ctypes.byref(d), stream_of(c)),
           flops=2.0 * m * n * k * batch,
           key=(m, n, k, batch, "AK" if a_kmajor else "AM", "BK" if b_kmajor else "BN", "a32" if a_f32 else "a16",
                split_k, flags))


def ln_fwd_prologue(gamma, beta, eps, *, mean=None, rstd=None, y_out=None):
    """LayerNorm of the GEMM's A rows inside lrce_gemm_ln (mode 1): the GEMM consumes LN(A); mean /
    rstd [m] and the normalised rows (y_out, f32) are written when given."""
    pro = N.LnPrologue()
    pro.mode, pro.gamma, pro.beta, pro.eps = 1, ptr(gamma), ptr(beta), float(eps)
    pro.mean, pro.rstd = ptr(mean), ptr(rstd)
    if y_out is not None:
        pro.y_out, pro.ld_y = ptr(y_out), y_out.shape[-1]
    return pro


def ln_bwd_prologue(x, mean, rstd, gamma, *, dgamma=None, dbeta=None, y_out=None, y2_out=None, drop=None):
    """LayerNorm backward of the GEMM's A rows (= dy) inside lrce_gemm_ln (mode 2): the GEMM consumes
    dropout_bwd(LN_bwd(dy)) (drop = (p, seed, group)); dx -> y_out, dropped dx -> y2_out, dgamma /
    dbeta accumulated (all optional)."""
    pro = N.LnPrologue()
    pro.mode, pro.gamma = 2, ptr(gamma)
    pro.x, pro.ld_x, pro.mean, pro.rstd = ptr(x), x.shape[-1], ptr(mean), ptr(rstd)
    pro.dgamma, pro.dbeta = ptr(dgamma), ptr(dbeta)
    if y_out is not None:
        pro.y_out, pro.ld_y = ptr(y_out), y_out.shape[-1]
    if y2_out is not None:
        pro.y2_out, pro.ld_y2 = ptr(y2_out), y2_out.shape[-1]
    if drop is not None and drop[0] > 0:
        pro.drop_p, pro.drop_seed, pro.drop_group = float(drop[0]), drop[1] & (2 ** 64 - 1), int(drop[2])
    return pro


def _split_for(m_out, n_out, k_red):
    """Split-K factor of a weight-gradient GEMM: ~2 blocks of 128x128 per CU, K slices >= 1024 deep."""
    tiles = math.ceil(m_out / 128) * math.ceil(n_out / 128)
    want = max(1, math.ceil(_SPLIT_PER_CU * NUM_CU / tiles))
    return int(max(1, min(want, k_red // _SPLIT_MIN_DEPTH)))


def _skinny_drop_ok(x, w, M, a_map=None):
    """Does lrce_gemm route this linear to the exact-f32 skinny kernel (the only one with the fused
    dropout epilogue)?  Mirrors the launcher's test: f32 A and W, K-major A, M <= 64, 16-B aligned."""
    return (x.dtype == F32 and w.dtype in (F32, F16) and M <= 64 and a_map is None and x.data_ptr() % 16 == 0
            and w.data_ptr() % (16 if w.dtype == F32 else 8) == 0)


def _glds_drop_ok(x, w, drop, a_map, c_map):
    """Does lrce_gemm take this 16-bit linear's fused dropout on the LDS-DMA path (element-wise mask,
    no row maps)?  Mirrors the launcher's test."""
    return (x.dtype in (F16, BF16) and w.dtype == x.dtype and int(drop[2]) == 1 and a_map is None and c_map is None
            and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0 and x.shape[-1] % 8 == 0)


def linear(x, w, bias=None, *, out=None, out_f32=False, gelu=False, pre_out=None, resid=None, c_map=None,
           a_map=None, rows=None, scale_cols=0, scale_val=1.0, row_scale=None, rows_per_scale=1, bf16_shadow=None,
           drop=None, ln=None):
    """y = x W^T (+b) [gelu] [*row_scale] [dropout] [+resid]; x [M,K] bf16/f32, W [N,K] bf16 (or f32:
    exact path).  drop = (p, seed, group): fused into the epilogue (exact-f32 skinny path, or the 16-bit
    LDS-DMA path with group 1), else a dropout launch."""
    f16 = x.dtype == F16
    M = rows if rows is not None else x.shape[0]
    if drop is not None and drop[0] > 0 and ln is None and not (_skinny_drop_ok(x, w, M, a_map) and c_map is None) \
            and not _glds_drop_ok(x, w, drop, a_map, c_map):
        y = linear(x, w, bias, out=out if resid is None else None, out_f32=out_f32, gelu=gelu, pre_out=pre_out,
                   c_map=c_map, a_map=a_map, rows=rows, scale_cols=scale_cols, scale_val=scale_val,
                   row_scale=row_scale, rows_per_scale=rows_per_scale)
        return dropout(y, drop[0], drop[1], out=out if out is not None else y, res=resid, group=drop[2])
    K = x.shape[-1]
    Nn = w.shape[0]
    flags = 0
    if bias is not None:
        flags |= N.EPI_BIAS
    if gelu:
        flags |= N.EPI_GELU
        if pre_out is not None:
            flags |= N.EPI_AUX_OUT | (N.EPI_AUX_F32 if pre_out.dtype == F32 else 0)
    if resid is not None:
        flags |= N.EPI_RESID
    if out is None:
        out = torch.empty((M if c_map is None else resid.shape[0] if resid is not None else M, Nn),
                          dtype=F32 if out_f32 else (F16 if f16 else BF16), device=x.device)
    if out.dtype == F32:
        flags |= N.EPI_OUT_F32
        if bf16_shadow is not None:
            flags |= N.EPI_OUT_BOTH
    aux = resid
    aux_out = pre_out if gelu else bf16_shadow
    gemm(x, w, out, M, Nn, K, flags=flags, bias=bias, aux=aux, ld_aux=Nn, aux_out=aux_out, ld_aux_out=Nn,
         a_map=a_map, c_map=c_map, scale_cols=scale_cols, scale_val=scale_val, row_scale=row_scale,
         rows_per_scale=rows_per_scale, drop=drop, f16=f16, ln=ln)
    return out


def linear_dx(dy, w, *, out=None, out_f32=True, dgelu_pre=None, a_map=None, rows=None, a_row_scale=None,
              a_rows_per_scale=1, accumulate=False, resid=None, drop=None, ln=None, alpha_dev=None):
    """dX = dY W (+ resid) ; dY [M,N] (bf16/f32), W [N,K] bf16 -> [M,K]; optional *gelu'(pre), and
    drop = (p, seed, group): the dropout backward mask (fused on the skinny path, else a launch).
    fp16 dY and W (the BERT backward): fp16 MFMAs, a 16-bit output is fp16; alpha_dev scales the
    product before the residual (the inverse gradient scale)."""
    M = rows if rows is not None else dy.shape[0]
    if drop is not None and drop[0] > 0 and ln is None and not (_skinny_drop_ok(dy, w, M, a_map) and not accumulate
                                                                and resid is None and a_row_scale is None):
        y = linear_dx(dy, w, out=out, out_f32=out_f32, dgelu_pre=dgelu_pre, a_map=a_map, rows=rows,
                      a_row_scale=a_row_scale, a_rows_per_scale=a_rows_per_scale, accumulate=accumulate, resid=resid,
                      alpha_dev=alpha_dev)
        return dropout_bwd(y, drop[0], drop[1], out=y, group=drop[2])
    Nn, K = w.shape
    flags = 0
    if dgelu_pre is not None:
        flags |= N.EPI_DGELU | (N.EPI_AUX_F32 if dgelu_pre.dtype == F32 else 0)
    if resid is not None:
        assert dgelu_pre is None
        flags |= N.EPI_RESID
    f16 = dy.dtype == F16 and w.dtype == F16
    if out is None:
        out = torch.empty((M, K), dtype=F32 if out_f32 else (F16 if f16 else BF16), device=dy.device)
    if out.dtype == F32:
        flags |= N.EPI_ACCUM if accumulate else N.EPI_OUT_F32
    gemm(dy, w, out, M, K, Nn, a_kmajor=True, b_kmajor=False, lda=_ld(dy), ldb=K, flags=flags,
         aux=dgelu_pre if dgelu_pre is not None else resid, ld_aux=K, a_map=a_map, a_row_scale=a_row_scale,
         a_rows_per_scale=a_rows_per_scale, drop=drop, ln=ln, f16=f16, alpha_dev=alpha_dev)
    return out


def linear_dw(dy, x, dw, *, a_map=None, rows=None, a_row_scale=None, a_rows_per_scale=1, bias_grad=None,
              alpha_dev=None):
    """dW[N,K] += dY^T X ; dY [M,N] (bf16/f32, rows optionally gathered by a_map), X [M,K] bf16.
    bias_grad: also db[N] += colsum(dY) (fused into the skinny f32 path, a column-sum launch otherwise).
    fp16 dY and X (the BERT backward): fp16 MFMAs; alpha_dev = the inverse gradient scale (device)."""
    M = rows if rows is not None else x.shape[0]
    Nn = dw.shape[0]
    K = dw.shape[1]
    split = _split_for(Nn, K, M)
    # one K slice: plain vector read-modify-write of the gradient (same stream => no race); split-K:
    # per-slice f32 slabs in a workspace + one reduce launch (bf16 operands), atomics otherwise
    flags = (N.EPI_ATOMIC if split > 1 else N.EPI_ACCUM) | (N.EPI_BIAS_GRAD if bias_grad is not None else 0)
    ws = None
    f16 = dy.dtype == F16 and x.dtype == F16
    if split > 1 and ((dy.dtype == BF16 and x.dtype == BF16) or f16):
        ws = torch.empty(split * Nn * K, dtype=F32, device=dw.device)
    gemm(dy, x, dw, Nn, K, M, a_kmajor=False, b_kmajor=False, lda=_ld(dy), ldb=_ld(x), ldc=K,
         flags=flags, bias=bias_grad, a_map=a_map, split_k=split, a_row_scale=a_row_scale,
         a_rows_per_scale=a_rows_per_scale, workspace=ws, f16=f16, alpha_dev=alpha_dev)


def linear_resid_ln(x, w, bias, resid, drop, gamma, beta, eps, split, *, out16=None, f16=True):
    """LN(resid + dropout(x W^T + bias)) for a deep-enough K: the GEMM's split-K slices as f32 slabs
    (LRCE_EPI_SLABS) and ONE lrce_splitk_reduce_ln launch (sum + bias + dropout + residual + LayerNorm).
    Returns (pre, y, mean, rstd): pre = the LayerNorm input (its backward reads it), y f32, and out16
    (optional) the fp16 (f16) / bf16 copy of y."""
    rows, Kd = x.shape
    n = w.shape[0]
    ws = torch.empty(split * rows * n, dtype=F32, device=x.device)
    gemm(x, w, ws, rows, n, Kd, flags=N.EPI_SLABS, split_k=split, workspace=ws, f16=f16)
    pre = torch.empty(rows, n, dtype=F32, device=x.device)
    y = torch.empty(rows, n, dtype=F32, device=x.device)
    mean = torch.empty(rows, dtype=F32, device=x.device)
    rstd = torch.empty(rows, dtype=F32, device=x.device)
    p, seed = (float(drop[0]), drop[1] & (2 ** 64 - 1)) if drop is not None and drop[0] > 0 else (0.0, 0)
    call("lrce_splitk_reduce_ln", ptr(ws), split, rows, n, ptr(bias), ptr(resid),
         resid.stride(0) if resid is not None else 0, p, seed, ptr(pre), ptr(gamma), ptr(beta), float(eps), ptr(y),
         ptr(out16), int(out16 is not None and out16.dtype == F16), ptr(mean), ptr(rstd), stream_of(y))
    return pre, y, mean, rstd


def linear_dw_batched(items, store=False):
    """dW_i += dY_i^T X_i (+ db_i += colsum(dY_i)) for items [(dy16, x16, dw, db|None)] of one shape
    (bf16 [T, out] / [T, in], f32 [out, in]).  store: dW_i = dY_i^T X_i (the gradients are known zero:
    FlatParams.claim_fresh); db_i still added.  (linear_dw_grouped with one shape.)"""
    dy0, x0, dw0, db0 = items[0]
    shape = (tuple(dy0.shape), tuple(x0.shape), db0 is not None)
    for dy, x, dw, db in items:
        if (tuple(dy.shape), tuple(x.shape), db is not None) != shape:
            raise N.NativeError("linear_dw_batched: items differ in shape")
    linear_dw_grouped([(dy, x, dw, db, store) for dy, x, dw, db in items])


def linear_dw_grouped(items, split=1):
    """Weight gradients of linears of any shapes over the same tokens, items [(dy16, x16, dw, db|None,
    store[, alpha_dev])] (bf16 or fp16 [T, out] / [T, in], f32 [out, in]): dW = (store) or += (not
    store) a dY^T X, db += a colsum(dY), a = alpha_dev[0] (a device f32, e.g. an inverse gradient scale)
    or 1, as grouped launches (lrce_gemm_grouped: every entry's tiles in one grid; fp16 and bf16
    entries in separate launches).  split > 1: each entry's K in `split` slices of a multiple of 64
    tokens, every slice storing f32 slabs (weight and bias), then ONE lrce_slab_sum_grouped launch sums
    them in slice order into dW / db (deterministic; the long-K stages whose few tiles would otherwise
    run one K loop each for milliseconds)."""
    T = items[0][1].shape[0]
    kc = 0
    if split > 1:
        kc = -(-(-(-T // split)) // 64) * 64
        split = -(-T // kc)
    dev = items[0][2].device
    if split > 1:
        wn = sum(it[2].numel() for it in items) * split
        bn = sum(it[2].shape[0] for it in items if it[3] is not None) * split
        wslab = torch.empty(wn, dtype=F32, device=dev)
        bslab = torch.zeros(max(bn, 4), dtype=F32, device=dev)
        sums = (N.SlabSum * (2 * len(items)))()
        nsum = wo = bo = 0
    arr = (N.GemmItem * len(items))()
    flops = 0.0
    for e, item in zip(arr, items):
        dy, x, dw, db, store = item[:5]
        al = item[5] if len(item) > 5 else None
        O, I = dw.shape
        if (dy.dtype not in (BF16, F16) or x.dtype != dy.dtype or dw.dtype != F32 or dy.shape != (T, O)
                or x.shape != (T, I) or not dw.is_contiguous() or dy.stride(1) != 1 or x.stride(1) != 1
                or (db is not None and (db.dtype != F32 or db.shape != (O,) or not db.is_contiguous()))
                or (al is not None and (al.dtype != F32 or al.device != dw.device))):
            raise N.NativeError("linear_dw_grouped: an item's dtype / shape / layout")
        e.a, e.b, e.alpha_dev = ptr(dy), ptr(x), ptr(al)
        e.m, e.n, e.lda, e.ldb, e.ldc = O, I, _ld(dy), _ld(x), I
        e.f16 = int(dy.dtype == F16)
        e.split, e.k_chunk = max(split, 1), kc
        if split > 1:
            e.c = wslab.data_ptr() + 4 * wo
            sums[nsum].slabs, sums[nsum].dst, sums[nsum].n = e.c, ptr(dw), O * I
            sums[nsum].split, sums[nsum].accumulate = split, int(not store)
            nsum += 1
            wo += O * I * split
            e.bias = None
            if db is not None:
                e.bias = bslab.data_ptr() + 4 * bo
                sums[nsum].slabs, sums[nsum].dst, sums[nsum].n = e.bias, ptr(db), O
                sums[nsum].split, sums[nsum].accumulate = split, 1
                nsum += 1
                bo += O * split
            e.flags = N.EPI_OUT_F32 | (N.EPI_BIAS_GRAD if db is not None else 0)
        else:
            e.c, e.bias = ptr(dw), ptr(db)
            e.flags = (N.EPI_OUT_F32 if store else N.EPI_ACCUM) | (N.EPI_BIAS_GRAD if db is not None else 0)
        flops += 2.0 * O * I * T
    dw0 = items[0][2]

    def run():
        call("lrce_gemm_grouped", arr, len(items), T, 1.0, stream_of(dw0))
        if split > 1:
            call("lrce_slab_sum_grouped", sums, nsum, stream_of(dw0))
    _timed("gemm", dw0, run, flops=flops, key=("grouped", T, len(items), split))


def colsum(x, out, *, row_map=None, rows=None, row_scale=None, rows_per_scale=1):
    M = rows if rows is not None else x.shape[0]
    call("lrce_colsum", ptr(x), int(x.dtype == F32), ptr(row_map), x.shape[-1], M, x.shape[-1], ptr(row_scale),
         rows_per_scale, ptr(out), stream_of(out))


def layernorm(x, w, b, eps, *, out=None, out_f32=False, in_map=None, nseg=1, out_map=None, rows=None, cols=None,
              stats=True, out_rows=None, bf16_copy=None):
    """bf16_copy: optional 16-bit copy of y (bf16, or torch.float16 for the fp16 BERT forward)."""
    R = rows if rows is not None else x.shape[0]
    Cc = cols if cols is not None else x.shape[-1] * nseg
    if out is None:
        out = torch.empty((out_rows or R, Cc), dtype=F32 if out_f32 else BF16, device=x.device)
    mean = torch.empty(R, dtype=F32, device=x.device) if stats else None
    rstd = torch.empty(R, dtype=F32, device=x.device) if stats else None
    call("lrce_layernorm_fwd", ptr(x), int(x.dtype == F32), ptr(in_map), nseg, ptr(w), ptr(b), eps, ptr(out),
         int(out.dtype == F32), ptr(bf16_copy), ptr(out_map), ptr(mean), ptr(rstd), R, Cc,
         int(bf16_copy is not None and bf16_copy.dtype == F16), stream_of(out))
    return out, mean, rstd


def layernorm_bwd(dy, x, mean, rstd, w, dx, *, dy_map=None, in_map=None, nseg=1, dres=None, dw=None, db=None,
                  rows=None, cols=None, dx16=None, dx16_map=None, dx_scale=None, dx_scale_rps=1, workspace=True,
                  defer=None):
    """dx16: optional bf16 copy of dx (times dx_scale[r / dx_scale_rps], at row dx16_map[r]).
    workspace=False: dw/db by per-block atomics instead of the two-pass partials sum.
    defer: a DeferredGrads — the dw / db reduction joins its batch (layernorm_grad_reduce at its flush)
    instead of a launch of its own.  dx may be None when dx16 is given (returns dx16 then)."""
    R = rows if rows is not None else mean.shape[0]
    Cc = cols if cols is not None else w.shape[0]
    out = dx if dx is not None else dx16
    ws, nws = None, 0
    if workspace and (dw is not None or db is not None):
        nws = N.lib().lrce_layernorm_bwd_workspace(R, Cc)
        ws = torch.empty(nws, dtype=F32, device=out.device) if nws > 0 else None
    args = (ptr(dy), int(dy.dtype == F32), ptr(dy_map), ptr(x), int(x.dtype == F32), ptr(in_map), nseg, ptr(mean),
            ptr(rstd), ptr(w), ptr(dx), ptr(dres), ptr(dw), ptr(db), R, Cc, ptr(dx16), ptr(dx16_map), ptr(dx_scale),
            dx_scale_rps, ptr(ws), nws)
    if defer is None or ws is None:
        call("lrce_layernorm_bwd", *args, stream_of(out))
        return out
    nb = ctypes.c_int(0)
    call("lrce_layernorm_bwd_deferred", *args, ctypes.byref(nb), stream_of(out))
    if nb.value > 0:
        defer.ln.append((ws, nb.value, Cc, dw, db))
    return out


class DeferredGrads:
    """Parameter-gradient reductions that nothing downstream reads before the optimizer, collected over
    several blocks and issued as batched launches by flush(): LayerNorm gamma / beta sums
    (layernorm_bwd(defer=...)) and relative-position bias-table gradients (wattn_dbias(defer=...)).
    Each sum is the one the immediate launch computes, in the same order (bit-identical)."""

    def __init__(self, n_items=1):
        self.ln, self.db, self.dw = [], [], []
        self.n_items = n_items   # blocks sharing this object (one weight gradient each per linear)

    def wants_dw(self, out_f, in_f, tokens):
        """Batch a weight gradient of this shape?  Only when each tile's single K loop stays short (one
        K slice per tile: a stage-1 weight, 282 240 tokens, would run its few workgroups for
        milliseconds) and the blocks' 128 x 128 tiles of this linear are a fair share of a chip-filling
        grouped launch (stage 4's 1024 x 1024 projection: 2 x 64)."""
        tiles = -(-out_f // 128) * -(-in_f // 128)
        if tokens > 32768:
            return True   # split-K slabs in the grouped launch (stages 1 and 2)
        return tiles * self.n_items >= 64

    def flush(self, stream_tensor):
        if self.dw:
            # every deferred weight gradient (the stage's linears x blocks, same tokens) in one grouped grid
            by_t = {}   # (blocks of a padded stage may differ in token count: one grid per count)
            for it in self.dw:
                by_t.setdefault((it[1].shape[0], it[0].dtype), []).append(it)
            for (T, _), items in by_t.items():
                split = 1
                if T > 32768:   # a few tiles over a long K: slices so the grid fills ~one round of the chip
                    tiles = sum(-(-it[2].shape[0] // 128) * -(-it[2].shape[1] // 128) for it in items)
                    split = max(2, min(64, round(512 / tiles)))
                linear_dw_grouped(items, split=split)
        if self.ln:
            n = len(self.ln)
            arr = lambda vals, t: (t * n)(*vals)  # noqa: E731
            call("lrce_layernorm_grad_reduce", ctypes.cast(arr([ptr(i[0]) for i in self.ln], ctypes.c_void_p), ctypes.c_void_p),
                 ctypes.cast(arr([i[1] for i in self.ln], ctypes.c_int32), ctypes.c_void_p),
                 ctypes.cast(arr([i[2] for i in self.ln], ctypes.c_int32), ctypes.c_void_p),
                 ctypes.cast(arr([ptr(i[3]) for i in self.ln], ctypes.c_void_p), ctypes.c_void_p),
                 ctypes.cast(arr([ptr(i[4]) for i in self.ln], ctypes.c_void_p), ctypes.c_void_p), n,
                 stream_of(stream_tensor))
        if self.db:
            n = len(self.db)
            arr = lambda vals, t: ctypes.cast((t * n)(*vals), ctypes.c_void_p)  # noqa: E731
            call("lrce_wattn_dbias_batched", arr([ptr(i[0]) for i in self.db], ctypes.c_void_p),
                 arr([i[1] for i in self.db], ctypes.c_int32), arr([i[2] for i in self.db], ctypes.c_int32),
                 arr([i[3] for i in self.db], ctypes.c_int32), arr([ptr(i[4]) for i in self.db], ctypes.c_void_p),
                 arr([ptr(i[5]) for i in self.db], ctypes.c_void_p), n, stream_of(stream_tensor))
        self.ln, self.db, self.dw = [], [], []


def scale_cast_bf16(x, row_scale=None, rows_per_scale=1, out=None):
    """bf16(x[r] * row_scale[r // rows_per_scale]) for a 2-D f32 x."""
    rows, cols = x.shape[0], x.shape[-1]
    if out is None:
        out = torch.empty(rows, cols, dtype=BF16, device=x.device)
    call("lrce_scale_cast_bf16", ptr(x), rows, cols, ptr(row_scale), rows_per_scale, ptr(out), stream_of(out))
    return out


def wattn_bias_elems(n_pat, nH):
    return N.lib().lrce_wattn_bias_elems(n_pat, nH)


def wattn_bias_build(table, index, n, nH, region, n_pat, bias_fwd, bias_bwd):
    """bias_fwd f32 (lrce_wattn_fwd_grouped) or fp16 (lrce_wattn_qkv_fwd); bias_bwd f32 or fp16."""
    if bias_fwd.dtype not in (torch.float32, F16) or bias_bwd.dtype not in (torch.float32, F16):
        raise N.NativeError("wattn_bias_build: bias tiles must be f32 or fp16")
    call("lrce_wattn_bias_build", ptr(table), ptr(index), index.shape[-1], n, nH, ptr(region), n_pat,
         ptr(bias_fwd), int(bias_fwd.dtype == F16), ptr(bias_bwd), int(bias_bwd.dtype == F16), stream_of(bias_fwd))


WATTN_GROUP = 4   # windows per workgroup of lrce_wattn_fwd_grouped


def wattn_groups(win_pat, n_win, device):
    """Group windows by mask pattern, WATTN_GROUP per group (lrce_wattn_fwd_grouped): returns
    (win_list int32 [n_groups*G] with -1 in empty slots | None for the identity, grp_pat | None, n_groups)."""
    G = WATTN_GROUP
    if win_pat is None:
        return None, None, (n_win + G - 1) // G
    wp = win_pat.detach().to("cpu", torch.int64)
    lists, pats = [], []
    for pat in torch.unique(wp).tolist():
        ids = torch.nonzero(wp == pat).flatten()
        pad = (-ids.numel()) % G
        ids = torch.cat([ids, torch.full((pad,), -1, dtype=torch.int64)])
        lists.append(ids)
        pats += [pat] * (ids.numel() // G)
    win_list = torch.cat(lists).to(torch.int32).to(device)
    grp_pat = torch.tensor(pats, dtype=torch.int32).to(device)
    return win_list, grp_pat, len(pats)


def wattn_fwd_grouped(qkv, bias_fwd, groups, out, lse, n_win, n, nH):
    # algorithmic bytes: Q, K, V read + O written, bf16: 8 n d per (window, head)
    win_list, grp_pat, n_groups = groups
    _timed("wattn_fwd", out, lambda: call("lrce_wattn_fwd_grouped", ptr(qkv), ptr(bias_fwd), ptr(win_list), ptr(grp_pat),
                                           n_groups, ptr(out), ptr(lse), n_win, n, nH, stream_of(out)),
           flops=4.0 * n * n * 32 * n_win * nH, nbytes=8.0 * n * 32 * n_win * nH, key=(n_win, nH))


def wattn_qkv_fwd(x, w_qkv, b_qkv, qscale, bias_fwd, win_pat, qkv, out, lse, n_win, n, nH, win_order=None):
    """Fused QKV projection + window attention forward (csrc/window_fused.hip).  Algorithmic work per
    launch: the QKV GEMM 2 * (n_win n) * C * 3C + attention 4 n^2 d per (window, head); bytes: x read,
    W_qkv read, qkv + out written (bf16)."""
    C = x.shape[-1]
    M = n_win * n
    _chk(x, BF16, "x"); _chk(w_qkv, BF16, "w_qkv"); _chk(qkv, BF16, "qkv"); _chk(out, BF16, "out")
    _chk(bias_fwd, F16, "bias_fwd")
    _timed("wattn_qkv_fwd", out, lambda: call("lrce_wattn_qkv_fwd", ptr(x), ptr(w_qkv), ptr(b_qkv), float(qscale),
                                               ptr(bias_fwd), ptr(win_pat), ptr(win_order), ptr(qkv), ptr(out),
                                               ptr(lse), n_win, n, nH, stream_of(out)),
           flops=2.0 * M * C * 3 * C + 4.0 * n * n * 32 * n_win * nH,
           nbytes=2.0 * (M * C + 3 * C * C + M * 3 * C + M * C), key=(n_win, nH))


def wattn_bwd(qkv, out, dout, lse, bias_bwd, win_pat, dqkv, dbias_part, n_win, n, nH, window):
    """One-kernel window-attention backward; window = (wd, wh, ww) with n = wd*wh*ww.  dbias_part (f32,
    wattn_dbias_part_elems) receives the bias-table gradient binned by relative position (wattn_dbias)."""
    _, wh, ww = window
    # algorithmic work: dV, dP, dQ, dK = 8 n^2 d per (window, head)
    if bias_bwd.dtype not in (torch.float32, F16):
        raise N.NativeError("wattn_bwd: bias tiles must be f32 or fp16")
    _timed("wattn_bwd", dqkv, lambda: call("lrce_wattn_bwd", ptr(qkv), ptr(out), ptr(dout), ptr(lse), ptr(bias_bwd),
                                            int(bias_bwd.dtype == F16), ptr(win_pat), ptr(dqkv), ptr(dbias_part),
                                            n_win, n, nH, wh, ww, stream_of(dqkv)),
           flops=8.0 * n * n * 32 * n_win * nH,
           nbytes=2.0 * n * 32 * n_win * nH * 8, key=(n_win, nH))


def frames_resize(frames, frame_idx, out_h=224, out_w=224, out=None):
    """frames uint8 [T, H, W, 3] (device), frame_idx int32 [n] (device, values < T) -> f32
    [n, 3, out_h, out_w]: Pillow-exact antialiased bilinear resample + ToTensor (csrc/video_io.hip)."""
    _chk(frames, torch.uint8, "frames")
    frames = frames.contiguous()
    _chk(frame_idx, torch.int32, "frame_idx")
    T, H, W, C = frames.shape
    if C != 3:
        raise N.NativeError("frames_resize: frames must be [T, H, W, 3] RGB")
    n = frame_idx.numel()
    if out is None:
        out = torch.empty(n, 3, out_h, out_w, device=frames.device)
    call("lrce_frames_resize", ptr(frames), T, H, W, ptr(frame_idx), n, out_h, out_w, ptr(out), stream_of(out))
    return out


def wattn_n_bins(window):
    wd, wh, ww = window
    return (2 * wd - 1) * (2 * wh - 1) * (2 * ww - 1)


def wattn_dbias_part_elems(n_win, nH, window):
    return N.lib().lrce_wattn_dbias_part_elems(n_win, nH, wattn_n_bins(window))


def wattn_bin_rows(index, window):
    """Table row of every relative-position bin of lrce_wattn_bwd (int32 [n_bins], -1 = unused, on
    index's device).  The kernel bins (query i, key j) at code(i) - code(j) + off with
    code(t, h, w) = (t (2wh-1) + h)(2ww-1) + w; the row is read from relative_position_index[:n, :n]
    itself (video_swin_ori.py:133-148, 171) and every pair of a bin must agree on it.  Built once per
    (block, geometry) on the host: the index is a constant buffer."""
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        raise RuntimeError("wattn_bin_rows: build the bias-gradient bin map before HIP-graph capture (run one eager step)")
    wd, wh, ww = window
    n = wd * wh * ww
    idx = index.detach().to("cpu", torch.int64)[:n, :n]
    x = torch.arange(n)
    code = ((x // (wh * ww)) * (2 * wh - 1) + (x // ww) % wh) * (2 * ww - 1) + x % ww
    off = ((wd - 1) * (2 * wh - 1) + (wh - 1)) * (2 * ww - 1) + (ww - 1)
    b = (code[:, None] - code[None, :] + off).reshape(-1)
    nb = wattn_n_bins(window)
    rows = torch.full((nb,), -1, dtype=torch.int64)
    rows[b] = idx.reshape(-1)
    if not torch.equal(rows[b], idx.reshape(-1)):
        raise ValueError("relative_position_index is not a function of the relative position within the window")
    return rows.to(torch.int32).to(index.device)


def wattn_dbias(dbias_part, n_win, nH, window, bin_row, table_grad, defer=None):
    """defer: a DeferredGrads — join its batched launch (the part buffer is kept until its flush)."""
    if defer is not None:
        defer.db.append((dbias_part, n_win, nH, wattn_n_bins(window), bin_row, table_grad))
        return
    call("lrce_wattn_dbias", ptr(dbias_part), n_win, nH, wattn_n_bins(window), ptr(bin_row), ptr(table_grad),
         stream_of(table_grad))


def mha_desc(q, Lq, *, k1, v1, lk1, ld_kv1, stride_kv1_b, kv1_bdiv=1, k2=None, v2=None, lk2=0, ld_kv2=0,
             stride_kv2_b=0, kv2_bdiv=1, key_mask=None, out, lse, B, H, scale, ld_q=None, ld_o=None, drop_p=0.0,
             seed=0, d=64):
    """q/k/v/out torch.float16 selects the fp16 forward (BERT); the backward reads bf16 tensors."""
    m = N.MhaDesc()
    m.q, m.ld_q = ptr(q), ld_q if ld_q is not None else H * d
    m.k1, m.v1, m.ld_kv1, m.stride_kv1_b, m.kv1_bdiv, m.lk1 = ptr(k1), ptr(v1), ld_kv1, stride_kv1_b, kv1_bdiv, lk1
    m.k2, m.v2, m.ld_kv2, m.stride_kv2_b, m.kv2_bdiv, m.lk2 = ptr(k2), ptr(v2), ld_kv2, stride_kv2_b, kv2_bdiv, lk2
    m.key_mask, m.out, m.ld_o, m.lse = ptr(key_mask), ptr(out), ld_o if ld_o is not None else H * d, ptr(lse)
    m.B, m.H, m.Lq, m.d, m.scale = B, H, Lq, d, scale
    m.drop_p, m.seed = float(drop_p), seed & (2 ** 64 - 1)
    m.f32_io = int(q.dtype == F32)
    m.f16 = int(q.dtype == F16)
    if (out.dtype == F32) != (q.dtype == F32):
        raise N.NativeError("mha: q and out must share dtype (bf16, or f32 for the decoder path)")
    return m


# ---- recurrent decoder: per-head fused attention blocks (csrc/decoder.hip) -------------------------
DEC_MAX_ROWS = 64
_DEC_WS = {}


def dec_workspace(device):
    """The hand-off slab + per-row arrival counters of the fused decoder blocks (one per device; the
    decoder runs on one stream at a time).  Allocated on first use (the eager warm-up step)."""
    key = torch.device(device)
    ws = _DEC_WS.get(key)
    if ws is None:
        slab = torch.empty(int(N.lib().lrce_dec_slab_elems(DEC_MAX_ROWS)), dtype=F32, device=key)
        ctr = torch.zeros(DEC_MAX_ROWS, dtype=torch.int32, device=key)
        _DEC_WS[key] = ws = (slab, ctr)
    return ws


# ---- recurrent decoder: one persistent launch per recurrent step (csrc/decoder_step.hip) ------------
_STEP_WS = {}
DEC_STEP_FWD_FIELDS = ("x0", "sad", "x1p", "x1", "q", "ctx", "x2p", "x2", "x3p", "pre", "gd", "lse",
                       "m1", "r1", "m2", "r2", "m3", "r3")
DEC_STEP_BWD_FIELDS = ("df", "dgp", "dcao", "dq", "dsao", "dsav", "dln1", "dln2", "dln3")


def dec_step_workspace(device):
    """(ws f32, counters int32, status int32[4]) of the persistent decoder step, one per device (the
    decoder runs on one stream at a time).  The workspace starts with every byte 0xFF: the hand-off
    buffers' sentinel, which every launch leaves in place (lrce_dec_step_reset restores it)."""
    key = torch.device(device)
    ws = _STEP_WS.get(key)
    if ws is None:
        L = N.lib()
        ws = (torch.full((int(L.lrce_dec_step_ws_elems()),), -1, dtype=torch.int32, device=key).view(F32),
              torch.zeros(int(L.lrce_dec_step_counter_words()), dtype=torch.int32, device=key),
              torch.zeros(4, dtype=torch.int32, device=key))
        _STEP_WS[key] = ws
    return ws


def dec_step_field(kind, field, layer, B, S, n_layers):
    """Element offset of an arena field (include/lrce_hip.h lrce_dec_step_field); field -1: the size."""
    names = DEC_STEP_BWD_FIELDS if kind else DEC_STEP_FWD_FIELDS
    f = names.index(field) if isinstance(field, str) else field
    off = int(N.lib().lrce_dec_step_field(kind, f, layer, B, S, n_layers))
    if off < 0:
        raise N.NativeError(f"dec_step_field({kind}, {field}, {layer}, B={B}, S={S}, L={n_layers})")
    return off


def dec_step_fwd(desc, stream_tensor):
    _timed("decoder", stream_tensor, lambda: call("lrce_dec_step_fwd", ctypes.byref(desc), stream_of(stream_tensor)))


def dec_step_bwd(desc, stream_tensor):
    _timed("decoder", stream_tensor, lambda: call("lrce_dec_step_bwd", ctypes.byref(desc), stream_of(stream_tensor)))


def dec_step_status(device, reset=True):
    """status[0] of the persistent decoder step (synchronises): 0, or the code of a hand-off that timed
    out (0x100-0x1FFF: phase << 8 | layer).  A timed-out launch leaves the hand-off buffers half used:
    reset=True re-arms them and zeroes the counters and the status."""
    ws = _STEP_WS.get(torch.device(device))
    if ws is None:
        return 0
    code = int(ws[2][0].item())
    if code and reset:
        call("lrce_dec_step_reset", ptr(ws[0]), ptr(ws[1]), ptr(ws[2]), stream_of(ws[2]))
        torch.cuda.synchronize(device)
    return code


def dec_kv(k1, *, stride1, ld1, bdiv1, lk1, k2=None, stride2=0, ld2=0, bdiv2=1, lk2=0, v_off):
    """Memory K/V of one recurrent step (bf16; V at K + v_off elements): key j < lk1 of query row b
    at k1[(b // bdiv1) * stride1 + j * ld1], the rest from k2 likewise."""
    kv = N.DecKv()
    kv.k1, kv.stride1, kv.ld1, kv.bdiv1, kv.lk1 = ptr(k1), stride1, ld1, bdiv1, lk1
    kv.k2, kv.stride2, kv.ld2, kv.bdiv2, kv.lk2 = ptr(k2), stride2, ld2, bdiv2, lk2 if k2 is not None else 0
    kv.v_off = v_off
    kv._keep = (k1, k2)
    return kv


def _dec_ws(a, device, p, seed):
    a.drop_p, a.seed = float(p), seed & (2 ** 64 - 1)
    slab, ctr = dec_workspace(device)
    a.slab, a.counters = ptr(slab), ptr(ctr)


def dec_sa_fwd(x_in, wv, bv, wo, bo, *, sad, x1p, p, seed, ln=None, eps=1e-12, x0_out=None, mean_out=None, rstd_out=None):
    """x1p = x0 + drop(out_proj(drop_head(v_proj(x0)))), x0 = LN(x_in) (ln = (gamma, beta)) or x_in."""
    a = N.DecSa()
    a.B, a.x_in = x_in.shape[0], ptr(x_in)
    if ln is not None:
        a.ln_gamma, a.ln_beta, a.eps = ptr(ln[0]), ptr(ln[1]), float(eps)
        a.x0_out, a.mean_out, a.rstd_out = ptr(x0_out), ptr(mean_out), ptr(rstd_out)
    a.wv, a.bv, a.wo, a.bo, a.sad, a.x1p = ptr(wv), ptr(bv), ptr(wo), ptr(bo), ptr(sad), ptr(x1p)
    _dec_ws(a, x_in.device, p, seed)
    _timed("decoder", x1p, lambda: call("lrce_dec_sa_fwd", ctypes.byref(a), stream_of(x1p)))


def dec_ca_fwd(x1p, g1, b1, wq, bq, kv, wo, bo, *, x1_out, mean_out, rstd_out, q_out, ctx_out, lse_out, x2p, p, seed,
               eps=1e-12):
    """x1 = LN1(x1p); ctx = attention(W_q x1 + b_q, memory); x2p = x1 + drop(out_proj(ctx)).  seed: the
    attention-dropout seed (the layer's seed + 2)."""
    a = N.DecCa()
    a.B, a.x1p, a.g1, a.b1, a.eps = x1p.shape[0], ptr(x1p), ptr(g1), ptr(b1), float(eps)
    a.x1_out, a.mean_out, a.rstd_out = ptr(x1_out), ptr(mean_out), ptr(rstd_out)
    a.wq, a.bq, a.kv = ptr(wq), ptr(bq), kv
    a.q_out, a.ctx_out, a.lse_out = ptr(q_out), ptr(ctx_out), ptr(lse_out)
    a.wo, a.bo, a.x2p = ptr(wo), ptr(bo), ptr(x2p)
    _dec_ws(a, x1p.device, p, seed)
    _timed("decoder", x2p, lambda: call("lrce_dec_ca_fwd", ctypes.byref(a), stream_of(x2p)))


def dec_ca_bwd(dx2, x2p, mean2, rstd2, g2, wo, kv, q, ctx, lse, wq, *, dcao_out, dq_out, dk1, dstride1, dld1, dx1_out, p,
               seed, dk2=None, dstride2=0, dld2=0, dv_off, dk2_store=False):
    """dk2_store: the text rows' dK / dV are written, not added (the backward's first recurrent step:
    the accumulation buffer needs no zeroing launch).  A bf16 dk1 (one writer per video row): the
    video rows' dK / dV are stored as bf16 directly (no f32 buffer + cast)."""
    a = N.DecCaBwd()
    a.B, a.dx2, a.x2p, a.mean2, a.rstd2, a.g2 = dx2.shape[0], ptr(dx2), ptr(x2p), ptr(mean2), ptr(rstd2), ptr(g2)
    a.dcao_out, a.wo, a.kv, a.q, a.ctx, a.lse = ptr(dcao_out), ptr(wo), kv, ptr(q), ptr(ctx), ptr(lse)
    if dk1.dtype == BF16:
        a.dq_out, a.dk1, a.dk1_bf16, a.dstride1, a.dld1 = ptr(dq_out), None, ptr(dk1), dstride1, dld1
    else:
        a.dq_out, a.dk1, a.dstride1, a.dld1 = ptr(dq_out), ptr(dk1), dstride1, dld1
    a.dk2, a.dstride2, a.dld2, a.dv_off = ptr(dk2), dstride2, dld2, dv_off
    a.wq, a.dx1_out = ptr(wq), ptr(dx1_out)
    a.dk2_store = int(bool(dk2_store))
    _dec_ws(a, dx2.device, p, seed)
    _timed("decoder", dx1_out, lambda: call("lrce_dec_ca_bwd", ctypes.byref(a), stream_of(dx1_out)))


def dec_sa_bwd(dx1, x1p, mean1, rstd1, g1, wo, wv, *, dsao_out, dsav_out, dx0_out, p, seed):
    a = N.DecSaBwd()
    a.B, a.dx1, a.x1p, a.mean1, a.rstd1, a.g1 = dx1.shape[0], ptr(dx1), ptr(x1p), ptr(mean1), ptr(rstd1), ptr(g1)
    a.dsao_out, a.wo, a.dsav_out, a.wv, a.dx0_out = ptr(dsao_out), ptr(wo), ptr(dsav_out), ptr(wv), ptr(dx0_out)
    _dec_ws(a, dx1.device, p, seed)
    _timed("decoder", dx0_out, lambda: call("lrce_dec_sa_bwd", ctypes.byref(a), stream_of(dx0_out)))


def dec_ln_grads(items, rows):
    """items: up to 3 (dy, x, mean, rstd, dgamma, dbeta) over `rows` rows of 768: dgamma += sum dy xhat,
    dbeta += sum dy (LayerNorm parameter gradients of every recurrent step at once); either of dgamma /
    dbeta may be None (frozen), not both."""
    n = len(items)
    arr = [(ctypes.c_void_p * 3)(*([ptr(it[k]) for it in items] + [None] * (3 - n))) for k in range(6)]
    st = items[0][4] if items[0][4] is not None else items[0][5]
    call("lrce_dec_ln_grads", *[ctypes.cast(a, ctypes.c_void_p) for a in arr], n, rows, stream_of(st))


def mha_fwd(desc, stream_tensor):
    call("lrce_mha_fwd", ctypes.byref(desc), stream_of(stream_tensor))


def mha_rebind(desc, *, q, k1, v1, out):
    """Point a forward descriptor at bf16 copies of its q / k / v / out (the backward of an fp16
    forward reads bf16)."""
    desc.q, desc.k1, desc.v1, desc.out = ptr(q), ptr(k1), ptr(v1), ptr(out)
    desc.f16 = 0
    return desc


def mha_bwd(desc, *, dout, dq, dk1, dv1, ld_dkv1, stride_dkv1_b, dk2=None, dv2=None, ld_dkv2=0, stride_dkv2_b=0,
            ld_dq=None, dkv1_store=False):
    """dkv1_store: the first segment's dK / dV rows are written, not accumulated (LrceMhaDesc).  fp16
    dq / dk1 / dv1 (with dkv1_store, the short self-attention path): the gradients are stored as fp16."""
    desc.dkv1_store = int(dkv1_store)
    desc.grad16 = int(dq.dtype == F16)
    if desc.grad16 and (dk1.dtype != F16 or dv1.dtype != F16 or not dkv1_store):
        raise N.NativeError("mha_bwd: fp16 gradients need fp16 dq / dk1 / dv1 and dkv1_store")
    desc.dout, desc.dq = ptr(dout), ptr(dq)
    desc.ld_dq = ld_dq if ld_dq is not None else desc.H * desc.d
    desc.dk1, desc.dv1, desc.ld_dkv1, desc.stride_dkv1_b = ptr(dk1), ptr(dv1), ld_dkv1, stride_dkv1_b
    desc.dk2, desc.dv2, desc.ld_dkv2, desc.stride_dkv2_b = ptr(dk2), ptr(dv2), ld_dkv2, stride_dkv2_b
    call("lrce_mha_bwd", ctypes.byref(desc), stream_of(dq))


def patch_im2col(clips, patches, *, layout="BSTCHW", normalize=True):
    """clips f32 (B,S,T,3,H,W) [layout BSTCHW] or (B,3,T,H,W) [layout BCTHW] -> patches bf16 [tokens, 96]."""
    if layout == "BSTCHW":
        B, S, T, C, H, W = clips.shape
        n, s_clip, s_t, s_c = B * S, T * C * H * W, C * H * W, H * W
    else:
        B, C, T, H, W = clips.shape
        n, s_clip, s_t, s_c = B, C * T * H * W, H * W, T * H * W
    call("lrce_patch_im2col", ptr(clips), n, T, H, W, s_clip, s_t, s_c, int(normalize), ptr(patches),
         stream_of(patches))


def slab_sum(items):
    """dst (=|+=) the sum of `split` consecutive slabs of n f32 each, in slab order, for every item
    (slabs, dst, n, split, accumulate) — one launch (lrce_slab_sum_grouped)."""
    if not items:
        return
    arr = (N.SlabSum * len(items))()
    for e, (slabs, dst, n, split, acc) in zip(arr, items):
        e.slabs, e.dst, e.n, e.split, e.accumulate = ptr(slabs), ptr(dst), int(n), int(split), int(acc)
    call("lrce_slab_sum_grouped", arr, len(items), stream_of(items[0][1]))


def cast_bf16(x, y):
    call("lrce_cast_bf16", ptr(x), ptr(y), x.numel(), stream_of(y))


def sum_shards_bf16(src, nshard, dst):
    """dst = bf16(sum of the nshard equal bf16 slices of src, in f32, in slice order)."""
    _chk(src, BF16, "src"); _chk(dst, BF16, "dst")
    if src.numel() != nshard * dst.numel():
        raise N.NativeError(f"sum_shards_bf16: {src.numel()} elements != {nshard} x {dst.numel()}")
    call("lrce_sum_shards_bf16", ptr(src), nshard, dst.numel(), ptr(dst), stream_of(dst))


def cast_f16(x, y):
    call("lrce_cast_f16", ptr(x), ptr(y), x.numel(), stream_of(y))


def cast_f16_bf16(x, y):
    _chk(x, F16, "x"); _chk(y, BF16, "y")
    call("lrce_cast_f16_bf16", ptr(x), ptr(y), x.numel(), stream_of(y))


def grad_scale(x, scale):
    """scale[0:2] = (S, 1/S), S a power of two with max|x| * S in [128, 256) (lrce_grad_scale);
    scale is a float32 [4] tensor zeroed once at allocation (scale[2:4] are the kernel's arrival words)."""
    _chk(x, F32, "x"); _chk(scale, F32, "scale")
    call("lrce_grad_scale", ptr(x), x.numel(), ptr(scale), stream_of(x))


def grad_scale_update(scales):
    """Delayed scales: every [S, 1/S, amax, -] slot of `scales` (f32, [..., 4]) with a recorded max
    becomes S = 2^(7 - floor(log2 max)), 1/S, the max cleared (lrce_grad_scale_update)."""
    _chk(scales, F32, "scales")
    call("lrce_grad_scale_update", ptr(scales), scales.numel() // 4, stream_of(scales))


def layernorm_bwd_f16s(dy, x, mean, rstd, w, dx, out16, scale, p, seed, *, dw=None, db=None, defer=None):
    """LayerNorm backward (f32 dy / x, identity maps) + out16 = fp16(scale[0] * dropout_bwd(dx)) in one
    launch, max|dx| recorded into scale[2] for grad_scale_update (lrce_layernorm_bwd_f16s).  defer: a
    DeferredGrads that takes the gamma / beta reduction (see layernorm_bwd)."""
    _chk(out16, F16, "out16"); _chk(scale, F32, "scale")
    R, Cc = mean.shape[0], w.shape[0]
    ws, nws = None, 0
    if dw is not None or db is not None:
        nws = N.lib().lrce_layernorm_bwd_workspace(R, Cc)
        ws = torch.empty(nws, dtype=F32, device=dy.device) if nws > 0 else None
    args = (ptr(dy), ptr(x), ptr(mean), ptr(rstd), ptr(w), ptr(dx), ptr(dw), ptr(db), R, Cc, ptr(out16), ptr(scale),
            float(p), seed & (2 ** 64 - 1), ptr(ws), nws)
    if defer is None or ws is None:
        call("lrce_layernorm_bwd_f16s", *args, stream_of(out16))
        return dx
    nb = ctypes.c_int(0)
    call("lrce_layernorm_bwd_f16s_deferred", *args, ctypes.byref(nb), stream_of(out16))
    if nb.value > 0:
        defer.ln.append((ws, nb.value, Cc, dw, db))
    return dx


def dropout_bwd_f16(dy, p, seed, scale, group=1, out=None):
    """fp16(scale[0] * dropout_bwd(dy)): the scaled fp16 GEMM operand of an f32 gradient."""
    if out is None:
        out = torch.empty(dy.shape, dtype=F16, device=dy.device)
    call("lrce_dropout_bwd_f16", ptr(dy), ptr(out), dy.numel(), float(p), seed & (2 ** 64 - 1), group, ptr(scale),
         stream_of(out))
    return out


def dropout(x, p, seed, out=None, out_bf16=None, res=None, group=1):
    """y = res + dropout(x) (train-mode nn.Dropout semantics, counter-hash mask)."""
    if out is None:
        out = torch.empty_like(x)
    call("lrce_dropout", ptr(x), ptr(res), ptr(out), ptr(out_bf16), x.numel(), float(p), seed & (2 ** 64 - 1), group,
         stream_of(out))
    return out


def dropout_bwd(dy, p, seed, out=None, group=1, out_bf16=None, f32=True):
    """dx = dy * keep / (1-p); out_bf16: also (or, f32=False: only) a bf16 copy for the GEMMs."""
    if out is None and f32:
        out = torch.empty_like(dy)
    if not f32:
        out = None
        if out_bf16 is None:
            out_bf16 = torch.empty(dy.shape, dtype=BF16, device=dy.device)
    call("lrce_dropout_bwd", ptr(dy), ptr(out), ptr(out_bf16), dy.numel(), float(p), seed & (2 ** 64 - 1), group,
         stream_of(dy))
    return out if f32 else out_bf16


def bert_embed_fwd(ids, types, word, pos, typ, out, rows, L, C):
    call("lrce_bert_embed_fwd", ptr(ids), ptr(types), ptr(word), ptr(pos), ptr(typ), ptr(out), rows, L, C, stream_of(out))


def bert_embed_bwd(dout, ids, types, dword, dpos, dtyp, rows, L, C, pad_id=0):
    call("lrce_bert_embed_bwd", ptr(dout), ptr(ids), ptr(types), ptr(dword), ptr(dpos), ptr(dtyp), rows, L, C, pad_id,
         stream_of(dout))


def video_posembed_fwd(x, cls, pos, len_, clip, out, B, S, Tg, P, C):
    call("lrce_video_posembed_fwd", ptr(x), ptr(cls), ptr(pos), ptr(len_), ptr(clip), ptr(out), B, S, Tg, P, C,
         stream_of(out))


def video_posembed_bwd(dout, dx, dcls, dpos, dlen, dclip, B, S, Tg, P, C, *, dx16=None):
    """dx (f32) and / or dx16 (bf16) may be None, not both; the table gradients are accumulated."""
    call("lrce_video_posembed_bwd", ptr(dout), ptr(dx), ptr(dx16), ptr(dcls), ptr(dpos), ptr(dlen), ptr(dclip), B, S, Tg,
         P, C, stream_of(dout))


def text_posembed_fwd(x, cls, pos, out, B, L, C):
    call("lrce_text_posembed_fwd", ptr(x), ptr(cls), ptr(pos), ptr(out), B, L, C, stream_of(out))


def text_posembed_bwd(dout, dx, dcls, dpos, B, L, C):
    call("lrce_text_posembed_bwd", ptr(dout), ptr(dx), ptr(dcls), ptr(dpos), B, L, C, stream_of(dout))


def l2norm_multi(p, chunk_tensor, n_chunks, sumsq, n_tensors, tensor_chunk_off=None, chunk_sq=None):
    call("lrce_l2norm_multi", ptr(p), ptr(chunk_tensor), n_chunks, ptr(sumsq), n_tensors, ptr(tensor_chunk_off),
         ptr(chunk_sq), stream_of(p))


def adamw_step(p, g, m, v, chunk_tensor, tensor_lr, sumsq, p_bf16, n_chunks, beta1, beta2, eps, wd, grad_scale, reg,
               bc1, bc2, step=None, sumsq_next=None, p_f16=None, f16_range=(0, 0), g_bf16=None, tensor_chunk_off=None,
               chunk_sq=None, n_tensors=None, skip=None):
    """step: optional f32 device scalar holding t (bias corrections computed on device: graph-safe).
    sumsq_next: optional [n_tensors] buffer receiving ||p_t||^2 of the updated parameters (zeroed first
    only without chunk_sq / tensor_chunk_off: the per-chunk path stores every entry).
    skip: optional (slots, c0, c1) — f32 gradient-scale slots [..., 4] whose found-inf words, when any is
    set, leave chunks [c0, c1) of this call unchanged (lrce_adamw_step)."""
    if skip is not None:
        _chk(skip[0], F32, "skip slots")
    call("lrce_adamw_step", ptr(p), ptr(g), ptr(m), ptr(v), ptr(chunk_tensor), ptr(tensor_lr), ptr(sumsq), ptr(p_bf16),
         n_chunks, beta1, beta2, eps, wd, grad_scale, reg, bc1, bc2, ptr(step), ptr(sumsq_next), ptr(p_f16),
         int(f16_range[0]), int(f16_range[1]), ptr(g_bf16), ptr(tensor_chunk_off), ptr(chunk_sq),
         (0 if tensor_chunk_off is None else tensor_chunk_off.numel() - 1) if n_tensors is None else n_tensors,
         *((None, 0, 0, 0) if skip is None else (ptr(skip[0]), skip[0].numel() // 4, int(skip[1]), int(skip[2]))),
         stream_of(p))


_RNG_OFFSETS = {}
_RNG_STRIDE = 0x2545F4914F6CDD1D & ((1 << 62) - 1)


def rng_offset(device):
    """The device RNG offset (int64 scalar) registered with lrce_set_rng_offset (one per process:
    the native library keeps a single pointer, so the first device registered wins)."""
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:   # "cuda" and "cuda:0" must name the same offset
        dev = torch.device("cuda", torch.cuda.current_device())
    t = _RNG_OFFSETS.get(dev)
    if t is None:
        t = torch.zeros(1, dtype=torch.int64, device=dev)
        _RNG_OFFSETS[dev] = t
        if len(_RNG_OFFSETS) == 1:
            call("lrce_set_rng_offset", ptr(t))
    return t


def rng_advance(device):
    """New masks for the next training step: one device add (captured into a graph it runs on every
    replay).  Forward and backward of one step see the same offset."""
    rng_offset(device).add_(_RNG_STRIDE)
