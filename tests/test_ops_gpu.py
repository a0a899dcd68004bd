"""Op-level parity of the HIP kernels (through the C ABI) against plain PyTorch fp32 references of
the same math.  GPU only."""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import lrce_oracle as O

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(0)


def K():
    from lrce import kernels
    return kernels


def rel(a, b):
    a = a.float(); b = b.float()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def bf(t):
    return t.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,Kd", [(256, 384, 128), (300, 200, 96), (1000, 768, 1024), (17, 72, 200)])
@pytest.mark.parametrize("a_km,b_km,a_f32", [(1, 1, 0), (1, 0, 0), (0, 0, 0), (1, 1, 1), (0, 0, 1), (0, 1, 0)])
def test_gemm_layouts(M, N, Kd, a_km, b_km, a_f32):
    k = K()
    A = torch.randn(M, Kd, device=dev)
    B = torch.randn(N, Kd, device=dev)
    if not a_km and M % 8:
        pytest.skip("M-major A needs M % 8 == 0")
    if not b_km and N % 8:
        pytest.skip("N-major B needs N % 8 == 0")
    Ab = A if a_f32 else bf(A)
    ref = bf(A).float() @ bf(B).float().t()
    a_store = Ab.contiguous() if a_km else Ab.t().contiguous()
    b_store = bf(B).contiguous() if b_km else bf(B).t().contiguous()
    C = torch.empty(M, N, device=dev, dtype=torch.float32)
    k.gemm(a_store, b_store, C, M, N, Kd, a_kmajor=bool(a_km), b_kmajor=bool(b_km), flags=16)
    torch.cuda.synchronize()
    assert rel(C, ref) < 2e-3


@pytest.mark.parametrize("M,N,Kd", [(17640, 512, 256), (17001, 520, 200)])
@pytest.mark.parametrize("b_km", [1, 0])
def test_gemm_tall_tiles(M, N, Kd, b_km):
    """Shapes whose 128x128 grid overshoots one round of the chip: the 192x128 tile path (ragged M,
    N and K tails included), with the bias + residual epilogue."""
    k = K()
    A = bf(torch.randn(M, Kd, device=dev))
    B = bf(torch.randn(N, Kd, device=dev))
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    b_store = B.contiguous() if b_km else B.t().contiguous()
    C = torch.empty(M, N, device=dev, dtype=torch.float32)
    k.gemm(A, b_store, C, M, N, Kd, a_kmajor=True, b_kmajor=bool(b_km), flags=16 | 1 | 8, bias=bias, aux=res, ld_aux=N)
    ref = A.float() @ B.float().t() + bias + res
    assert rel(C, ref) < 2e-3


@pytest.mark.parametrize("M,N,Kd", [(20000, 512, 128), (5003, 264, 64), (4100, 1024, 96), (3000, 512, 512)])
def test_gemm_short_k_prefetched_epilogues(M, N, Kd):
    """Short K (<= 8 full K tiles): every K tile issued up front when it has a stage of its own, and the
    epilogue's dGELU pre-activation / f32 residual loaded before the tiles.  dX = dY W with dGELU
    (bf16 out) and Y = X W^T + b + residual (f32 out, through a scatter map with dropped rows);
    ragged M, a K tail (96) and N % 8 != 0 columns (scalar epilogue) included."""
    k = K()
    dy = bf(torch.randn(M, Kd, device=dev))
    W = bf(torch.randn(Kd, N, device=dev) / math.sqrt(Kd))       # dX [M, N] = dY [M, Kd] W [Kd, N] (B N-major)
    pre = bf(torch.randn(M, N, device=dev))
    out = k.linear_dx(dy, W, out_f32=False, dgelu_pre=pre)
    g = pre.float()
    phi = 0.5 * (1 + torch.erf(g / math.sqrt(2)))
    ref = (dy.float() @ W.float()) * (phi + g * torch.exp(-0.5 * g * g) / math.sqrt(2 * math.pi))
    assert rel(out, ref) < 1e-2
    x = bf(torch.randn(M, Kd, device=dev))
    w = bf(torch.randn(N, Kd, device=dev) / math.sqrt(Kd))
    b = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    perm = torch.randperm(M, device=dev).int()
    perm[::7] = -1                                               # rows with no output (padded windows)
    y = torch.full((M, N), 7.0, device=dev)
    k.linear(x, w, b, out=y, resid=res, c_map=perm)
    ref = torch.full((M, N), 7.0, device=dev)
    keep = perm >= 0
    dst = perm[keep].long()
    ref[dst] = (x.float() @ w.float().t() + b)[keep] + res[dst]    # the residual is read at the output row
    assert rel(y, ref) < 2e-3


@pytest.mark.parametrize("M,N,Kd", [(320, 768, 768), (1800, 3072, 768), (300, 768, 3072), (17640, 512, 256)])
def test_gemm_f16_forward(M, N, Kd):
    """fp16 operands (the BERT forward, reference fp16 autocast): f16 MFMA, bias + GELU with the fp16
    pre-activation, fp16 and f32 outputs; the 64x64, 128x128 and tall tiles all have an f16 form."""
    k = K()
    h = torch.float16
    A = torch.randn(M, Kd, device=dev).to(h)
    B = (torch.randn(N, Kd, device=dev) / math.sqrt(Kd)).to(h)
    bias = torch.randn(N, device=dev)
    ref_pre = A.double() @ B.double().t() + bias.double()
    pre = torch.empty(M, N, device=dev, dtype=h)
    g = k.linear(A, B, bias, gelu=True, pre_out=pre)
    assert g.dtype == h and pre.dtype == h
    assert rel(pre, ref_pre.float()) < 1e-3          # fp16 storage: 2^-11 relative
    assert rel(g, F.gelu(ref_pre).float()) < 1e-3
    y = k.linear(A, B, bias, out_f32=True)
    assert rel(y, ref_pre.float()) < 1e-5            # exact products, f32 accumulation
    with pytest.raises(Exception):
        k.linear(A, B.to(torch.bfloat16), bias)      # mixed encodings are rejected


@pytest.mark.parametrize("bf", [False, True])
def test_gemm_batched_bias_stride(bf):
    """batch > 1 with a per-batch bias (stride_bias): BERT's query / key / value linears as one launch
    over weights and biases at one stride in the flat buffers (text.py _qkv); fp16 and bf16 forms."""
    k = K()
    h = torch.bfloat16 if bf else torch.float16
    M, N, Kd, gap = 320, 768, 768, 1024
    stride = N * Kd + gap
    wbuf = (torch.randn(3 * stride, device=dev) / math.sqrt(Kd)).to(h)
    bbuf = torch.randn(3 * stride, device=dev)
    A = torch.randn(M, Kd, device=dev).to(h)
    out = torch.empty(3, M, N, device=dev, dtype=h)
    k.gemm(A, wbuf, out, M, N, Kd, flags=k.N.EPI_BIAS, bias=bbuf, batch=3, stride_b=stride, stride_c=M * N,
           stride_bias=stride, f16=not bf)
    for i in range(3):
        W = wbuf[i * stride:i * stride + N * Kd].view(N, Kd)
        ref = A.double() @ W.double().t() + bbuf[i * stride:i * stride + N].double()
        assert rel(out[i], ref.float()) < (8e-3 if bf else 1e-3), i
    # a negative C stride (the reverse parameter layout of training: batch i writes plane 2 - i)
    out2 = torch.empty(3, M, N, device=dev, dtype=h)
    k.gemm(A, wbuf, out2[2], M, N, Kd, flags=k.N.EPI_BIAS, bias=bbuf, batch=3, stride_b=stride, stride_c=-M * N,
           stride_bias=stride, f16=not bf)
    assert torch.equal(out2.flip(0), out)
    # the weight-gradient form: dW_i += dY_i^T X, db_i += colsum(dY_i) (M-major A, one K slice)
    dy = torch.randn(3, M, N, device=dev).to(h)
    gw = torch.randn(3 * stride, device=dev)
    g0 = gw.clone()
    k.gemm(dy[0], A, gw, N, Kd, M, a_kmajor=False, b_kmajor=False, lda=N, ldb=Kd, ldc=Kd,
           flags=k.N.EPI_ACCUM | k.N.EPI_BIAS_GRAD, bias=gw[N * Kd:], batch=3, stride_a=M * N, stride_c=stride,
           stride_bias=stride, f16=not bf)
    for i in range(3):
        o = i * stride
        refw = g0[o:o + N * Kd].view(N, Kd).double() + dy[i].double().t() @ A.double()
        refb = g0[o + N * Kd:o + N * Kd + N].double() + dy[i].double().sum(0)
        assert rel(gw[o:o + N * Kd].view(N, Kd), refw.float()) < 1e-5, i
        assert rel(gw[o + N * Kd:o + N * Kd + N], refb.float()) < 1e-5, i
        assert torch.equal(gw[o + N * Kd + N:o + stride], g0[o + N * Kd + N:o + stride])   # the gap untouched


def test_f16_casts():
    k = K()
    x = torch.randn(1000, 768, device=dev) * 3
    h = torch.empty(x.shape, device=dev, dtype=torch.float16)
    k.cast_f16(x, h)
    assert torch.equal(h, x.to(torch.float16))
    b = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    k.cast_f16_bf16(h, b)
    assert torch.equal(b, h.float().to(torch.bfloat16))


@pytest.mark.parametrize("L", [32, 40])
def test_mha_self_f16_forward(L):
    """BERT self-attention with fp16 q/k/v/out: vs an fp64 reference of HF's masked SDPA."""
    k = K()
    B, H, D = 6, 12, 64
    q, kk, v = (torch.randn(B * L, H * D, device=dev).to(torch.float16) for _ in range(3))
    mask = torch.ones(B, L, dtype=torch.int32, device=dev)
    mask[:, 20:] = 0
    out = torch.empty(B * L, H * D, device=dev, dtype=torch.float16)
    lse = torch.empty(B, H, L, device=dev)
    desc = k.mha_desc(q, L, k1=kk, v1=v, lk1=L, ld_kv1=H * D, stride_kv1_b=L * H * D, key_mask=mask, out=out, lse=lse,
                      B=B, H=H, scale=0.125)
    k.mha_fwd(desc, out)
    qh, kh, vh = (t.double().view(B, L, H, D).transpose(1, 2) for t in (q, kk, v))
    s = qh @ kh.transpose(-1, -2) * 0.125 + (1 - mask.double())[:, None, None, :] * -1e30
    ref = (s.softmax(-1) @ vh).transpose(1, 2).reshape(B * L, H * D)
    assert rel(out, ref.float()) < 2e-3


def test_grad_scale_and_f16_operand():
    """lrce_grad_scale: S = 2^(7 - floor(log2 max|x|)) (1 for zeros / non-finite), 1/S, arrival words
    left zero (replayable); dropout_bwd_f16 = fp16(S * dropout_bwd)."""
    k = K()
    sc = torch.zeros(4, device=dev)
    for amax in (3.0e-6, 0.75, 1.0, 5.0e3):
        x = torch.randn(320 * 768, device=dev)
        x = x / x.abs().max() * amax
        k.grad_scale(x, sc)
        torch.cuda.synchronize()
        S = 2.0 ** (7 - math.floor(math.log2(amax)))
        assert float(sc[0]) == S and float(sc[1]) == 1.0 / S, (amax, sc)
        assert float(sc[2]) == 0.0 and float(sc[3]) == 0.0
        assert 128.0 <= amax * S < 256.0
        h = k.dropout_bwd_f16(x, 0.0, 0, sc)
        assert torch.equal(h, (x * S).to(torch.float16))
        hd = k.dropout_bwd_f16(x, 0.1, 7, sc)
        ref = k.dropout_bwd(x, 0.1, 7)
        assert rel(hd.float(), ref * S) < 1e-3
    for bad in (torch.zeros(4096, device=dev), torch.full((4096,), float("nan"), device=dev)):
        k.grad_scale(bad, sc)
        torch.cuda.synchronize()
        assert float(sc[0]) == 1.0 and float(sc[3]) == 0.0


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_layernorm_bwd_f16s_matches_unfused(p):
    """The BERT backward's fused LN backward + scaled fp16 operand (lrce_layernorm_bwd_f16s, delayed
    scale): dx, dw, db and the fp16 operand bit-identical to layernorm_bwd + dropout_bwd_f16 with the
    same scale; the slot records max|dx| and grad_scale_update turns it into the next scale."""
    k = K()
    k.rng_offset(dev).zero_()
    R, C = 320, 768
    x = torch.randn(R, C, device=dev) * 2 + 0.5
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev)
    _, mean, rstd = k.layernorm(x, g, b, 1e-12, out_f32=True)
    dy = torch.randn(R, C, device=dev) * 1e-3
    S = 2.0 ** 17
    dx = torch.empty(R, C, device=dev)
    dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    k.layernorm_bwd(dy, x, mean, rstd, g, dx, dw=dw, db=db)
    sc = torch.tensor([S, 1.0 / S, 0.0, 0.0], device=dev)
    ref16 = k.dropout_bwd_f16(dx, p, 41, sc)
    dx2 = torch.empty(R, C, device=dev)
    out16 = torch.empty(R, C, device=dev, dtype=torch.float16)
    dw2, db2 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    k.layernorm_bwd_f16s(dy, x, mean, rstd, g, dx2, out16, sc, p, 41, dw=dw2, db=db2)
    torch.cuda.synchronize()
    assert torch.equal(dx2, dx) and torch.equal(out16, ref16) and torch.equal(dw2, dw) and torch.equal(db2, db)
    amax = float(dx.abs().max())
    assert sc[2:3].view(torch.int32).item() == torch.tensor([amax]).view(torch.int32).item()
    k.grad_scale_update(sc)
    torch.cuda.synchronize()
    S2 = 2.0 ** (7 - math.floor(math.log2(amax)))
    assert float(sc[0]) == S2 and float(sc[1]) == 1.0 / S2 and float(sc[2]) == 0.0
    k.grad_scale_update(sc)                      # no recorded max: the scale stays
    torch.cuda.synchronize()
    assert float(sc[0]) == S2
    assert float(sc[3]) == 0.0                   # nothing overflowed: no found-inf flag


def test_found_inf_flag_skips_the_guarded_chunks():
    """An fp16 operand that overflows under its delayed scale (lrce_layernorm_bwd_f16s with S far above
    2^7 / max|dx|) raises the slot's found-inf word; lrce_adamw_step then leaves the guarded chunk range
    (parameters, moments) as it was and updates the rest, still writing every chunk's norm;
    lrce_grad_scale_update clears the flag and the next update runs in full (GradScaler's skipped step,
    agent_oe.py:40-42, for the group those operands feed)."""
    k = K()
    R, C = 320, 768
    x = torch.randn(R, C, device=dev)
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    _, mean, rstd = k.layernorm(x, g, b, 1e-12, out_f32=True)
    dy = torch.randn(R, C, device=dev)
    slots = torch.tensor([[2.0 ** 4, 2.0 ** -4, 0.0, 0.0], [2.0 ** 20, 2.0 ** -20, 0.0, 0.0]], device=dev)
    out16 = torch.empty(R, C, device=dev, dtype=torch.float16)
    dx = torch.empty(R, C, device=dev)
    k.layernorm_bwd_f16s(dy, x, mean, rstd, g, dx, out16, slots[0], 0.0, 3)
    torch.cuda.synchronize()
    assert float(slots[0, 3]) == 0.0 and bool(torch.isfinite(out16).all())
    k.layernorm_bwd_f16s(dy, x, mean, rstd, g, dx, out16, slots[1], 0.0, 3)   # |dx| 2^20 > 65504
    torch.cuda.synchronize()
    assert float(slots[1, 3]) != 0.0 and not bool(torch.isfinite(out16).all())
    n = 4 * 1024
    p = torch.randn(n, device=dev)
    gr = torch.randn(n, device=dev)
    m, v = torch.full((n,), 0.1, device=dev), torch.full((n,), 0.2, device=dev)
    p0, m0, v0 = p.clone(), m.clone(), v.clone()
    ct = torch.zeros(4, dtype=torch.int32, device=dev)
    lrs, chunk_sq = torch.tensor([1e-3], device=dev), torch.zeros(4, device=dev)
    sumsq_next = torch.zeros(1, device=dev)
    k.adamw_step(p, gr, m, v, ct, lrs, None, None, 4, 0.9, 0.999, 1e-8, 0.01, 1.0, 0.0, 0.1, 0.001,
                 sumsq_next=sumsq_next, chunk_sq=chunk_sq, n_tensors=0, skip=(slots, 1, 3))
    torch.cuda.synchronize()
    kept = slice(1024, 3 * 1024)
    assert torch.equal(p[kept], p0[kept]) and torch.equal(m[kept], m0[kept]) and torch.equal(v[kept], v0[kept])
    for c in (0, 3):
        sl = slice(c * 1024, (c + 1) * 1024)
        assert (p[sl] != p0[sl]).float().mean().item() > 0.99
    assert torch.allclose(chunk_sq, (p.view(4, 1024) ** 2).sum(1), rtol=1e-5)
    k.grad_scale_update(slots)
    torch.cuda.synchronize()
    assert float(slots[0, 3]) == 0.0 and float(slots[1, 3]) == 0.0
    p1 = p.clone()
    k.adamw_step(p, gr, m, v, ct, lrs, None, None, 4, 0.9, 0.999, 1e-8, 0.01, 1.0, 0.0, 0.1, 0.001, skip=(slots, 1, 3))
    torch.cuda.synchronize()
    assert (p[kept] != p1[kept]).float().mean().item() > 0.99


@pytest.mark.parametrize("M,N,Kd", [(320, 768, 768), (320, 3072, 768), (2000, 768, 3072)])
def test_gemm_f16_backward_layouts(M, N, Kd):
    """The fp16 BERT backward GEMMs: dX = dY W (B N-major) with dGELU or residual epilogues, dW = dY^T X
    (both M/N-major) with the fused bias gradient, alpha read from device memory."""
    k = K()
    h = torch.float16
    dy = (torch.randn(M, N, device=dev) * 100).to(h)          # a scaled gradient
    W = (torch.randn(N, Kd, device=dev) / math.sqrt(Kd)).to(h)
    X = torch.randn(M, Kd, device=dev).to(h)
    inv = torch.tensor([1.0 / 128], device=dev)
    res = torch.randn(M, Kd, device=dev)
    dx = k.linear_dx(dy, W, resid=res, alpha_dev=inv)
    ref = (dy.double() @ W.double()) / 128 + res.double()
    assert rel(dx, ref.float()) < 1e-5
    pre = torch.randn(M, Kd, device=dev).to(h)
    dg = k.linear_dx(dy, W, out_f32=False, dgelu_pre=pre)
    x = pre.double().requires_grad_(True)
    gg = torch.autograd.grad((F.gelu(x) * (dy.double() @ W.double())).sum(), x)[0]
    assert dg.dtype == h and rel(dg, gg.float()) < 2e-3
    dw = torch.zeros(N, Kd, device=dev)
    db = torch.zeros(N, device=dev)
    k.linear_dw(dy, X, dw, bias_grad=db, alpha_dev=inv)
    assert rel(dw, ((dy.double().t() @ X.double()) / 128).float()) < 1e-5
    assert rel(db, (dy.double().sum(0) / 128).float()) < 1e-5


@pytest.mark.parametrize("L", [32, 40])
def test_mha_self_f16_backward(L):
    """BERT self-attention backward with fp16 q/k/v/out and a scaled fp16 dout (the fp16 BERT
    backward): vs fp64 autograd of masked SDPA; dK / dV stored (dkv1_store) into NaN-filled buffers."""
    k = K()
    B, H, D = 6, 12, 64
    q, kk, v = (torch.randn(B * L, H * D, device=dev).to(torch.float16) for _ in range(3))
    mask = torch.ones(B, L, dtype=torch.int32, device=dev)
    mask[:, 20:] = 0
    out = torch.empty(B * L, H * D, device=dev, dtype=torch.float16)
    lse = torch.empty(B, H, L, device=dev)
    desc = k.mha_desc(q, L, k1=kk, v1=v, lk1=L, ld_kv1=H * D, stride_kv1_b=L * H * D, key_mask=mask, out=out, lse=lse,
                      B=B, H=H, scale=0.125)
    k.mha_fwd(desc, out)
    do = torch.randn(B * L, H * D, device=dev)
    S = 256.0
    dq, dk_, dv = (torch.full((B * L, H * D), float("nan"), device=dev) for _ in range(3))
    k.mha_bwd(desc, dout=(do * S).to(torch.float16), dq=dq, dk1=dk_, dv1=dv, ld_dkv1=H * D, stride_dkv1_b=L * H * D,
              dkv1_store=True)
    qh, kh, vh = (t.double().view(B, L, H, D).transpose(1, 2).requires_grad_(True) for t in (q, kk, v))
    s = qh @ kh.transpose(-1, -2) * 0.125 + (1 - mask.double())[:, None, None, :] * -1e30
    o = (s.softmax(-1) @ vh).transpose(1, 2).reshape(B * L, H * D)
    gq, gk, gv = torch.autograd.grad(o, (qh, kh, vh), do.double() * S)
    for got, ref in ((dq, gq), (dk_, gk), (dv, gv)):
        ref = ref.transpose(1, 2).reshape(B * L, H * D).float()
        assert torch.isfinite(got).all() and rel(got, ref) < 1e-2


@pytest.mark.parametrize("h", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,N,Kd", [(320, 768, 768), (320, 768, 3072), (1000, 264, 96), (9000, 512, 128)])
def test_fused_dropout_lds_dma_epilogue(h, M, N, Kd):
    """16-bit linears with nn.Dropout + residual fused into the LDS-DMA GEMM epilogue (the BERT
    residual branches, text.py _LayerFn): the same bits as GEMM + lrce_dropout (mask over the
    contiguous [M][N] result), 64x64 and 128x128 tile paths."""
    k = K()
    k.rng_offset(dev).zero_()
    x = torch.randn(M, Kd, device=dev).to(h)
    w = (torch.randn(N, Kd, device=dev) / math.sqrt(Kd)).to(h)
    b = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    for p in (0.1, 0.5):
        fused = k.linear(x, w, b, out_f32=True, resid=res, drop=(p, 91, 1))
        ref = k.dropout(k.linear(x, w, b, out_f32=True), p, 91, res=res)
        assert torch.equal(fused, ref), p
    k.rng_offset(dev).add_(12345)          # the device RNG offset moves the mask in both forms
    fused = k.linear(x, w, b, out_f32=True, resid=res, drop=(0.1, 91, 1))
    assert torch.equal(fused, k.dropout(k.linear(x, w, b, out_f32=True), 0.1, 91, res=res))
    k.rng_offset(dev).zero_()


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gemm_splitk_epilogue_reduce(p):
    """Split-K with the bias / dropout / residual epilogue applied by the reduce launch (the K = 3072
    BERT output projection): the dropout mask is lrce_dropout's (same zero pattern), values agree with
    the unsplit fused GEMM to f32 summation-order rounding."""
    k = K()
    k.rng_offset(dev).zero_()
    h = torch.float16
    M, N, Kd = 320, 768, 3072
    x = torch.randn(M, Kd, device=dev).to(h)
    w = (torch.randn(N, Kd, device=dev) / math.sqrt(Kd)).to(h)
    b = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    drop = (p, 93, 1) if p > 0 else None
    out = torch.empty(M, N, device=dev)
    ws = torch.empty(4 * M * N, device=dev)
    k.gemm(x, w, out, M, N, Kd, flags=k.N.EPI_BIAS | k.N.EPI_RESID | k.N.EPI_OUT_F32, bias=b, aux=res, ld_aux=N,
           split_k=4, workspace=ws, drop=drop, f16=True)
    ref = k.dropout(k.linear(x, w, b, out_f32=True), p, 93, res=res) if p > 0 else k.linear(x, w, b, out_f32=True, resid=res)
    assert torch.equal(out == res, ref == res)            # the same dropped elements
    assert rel(out - res, ref - res) < 1e-5


def test_gemm_batched_alpha_stride():
    """Batched weight-gradient GEMMs with a per-batch device alpha (stride_alpha): the deferred BERT
    weight gradients of all layers in one launch, each scaled by its own layer's 1/S; negative A / alpha
    strides (batches in ascending gradient address, layers in reverse)."""
    k = K()
    h = torch.float16
    nb, M, N, Kd, gap = 4, 320, 768, 3072, 512
    sg = N * Kd + N + gap                              # gradient slot per batch: weight, bias, gap
    dy = (torch.randn(nb, M, N, device=dev) * 64).to(h)
    X = torch.randn(nb, M, Kd, device=dev).to(h)
    alpha = torch.zeros(nb, 2, 4, device=dev)
    alpha[:, 0, 1] = torch.tensor([1 / 64, 1 / 128, 1 / 32, 1 / 256], device=dev)
    g = torch.randn(nb * sg, device=dev)
    g0 = g.clone()
    # batch i <-> operand plane nb-1-i (negative operand / alpha strides)
    k.gemm(dy[nb - 1], X[nb - 1], g, N, Kd, M, a_kmajor=False, b_kmajor=False, lda=N, ldb=Kd, ldc=Kd,
           flags=k.N.EPI_ACCUM | k.N.EPI_BIAS_GRAD, bias=g[N * Kd:], batch=nb, stride_a=-M * N, stride_b=-M * Kd,
           stride_c=sg, stride_bias=sg, f16=True, alpha_dev=alpha[nb - 1, 0, 1:2], stride_alpha=-8)
    for i in range(nb):
        j = nb - 1 - i
        a = float(alpha[j, 0, 1])
        o = i * sg
        refw = g0[o:o + N * Kd].view(N, Kd).double() + a * (dy[j].double().t() @ X[j].double())
        refb = g0[o + N * Kd:o + N * Kd + N].double() + a * dy[j].double().sum(0)
        assert rel(g[o:o + N * Kd].view(N, Kd), refw.float()) < 1e-5, i
        assert rel(g[o + N * Kd:o + N * Kd + N], refb.float()) < 1e-5, i
        assert torch.equal(g[o + N * Kd + N:o + sg], g0[o + N * Kd + N:o + sg])


@pytest.mark.parametrize("L", [32, 40])
def test_mha_self_f16_backward_fp16_gradients(L):
    """grad16: dq / dk / dv stored as fp16 column blocks of one [rows, 3 * 768] operand (the fused BERT
    q/k/v input-gradient GEMM): the bits of the f32 outputs cast to fp16."""
    k = K()
    B, H, D = 6, 12, 64
    C = H * D
    q, kk, v = (torch.randn(B * L, C, device=dev).to(torch.float16) for _ in range(3))
    mask = torch.ones(B, L, dtype=torch.int32, device=dev)
    mask[:, 25:] = 0
    out = torch.empty(B * L, C, device=dev, dtype=torch.float16)
    lse = torch.empty(B, H, L, device=dev)
    desc = k.mha_desc(q, L, k1=kk, v1=v, lk1=L, ld_kv1=C, stride_kv1_b=L * C, key_mask=mask, out=out, lse=lse,
                      B=B, H=H, scale=0.125, drop_p=0.1, seed=5)
    k.mha_fwd(desc, out)
    do = (torch.randn(B * L, C, device=dev) * 200).to(torch.float16)
    f = [torch.empty(B * L, C, device=dev) for _ in range(3)]
    k.mha_bwd(desc, dout=do, dq=f[0], dk1=f[1], dv1=f[2], ld_dkv1=C, stride_dkv1_b=L * C, dkv1_store=True)
    g = torch.full((B * L, 3 * C), float("nan"), device=dev, dtype=torch.float16)
    cols = (2 * C, C, 0)                       # dq, dk, dv blocks in the reverse (value, key, query) order
    k.mha_bwd(desc, dout=do, dq=g[:, cols[0]:cols[0] + C], dk1=g[:, cols[1]:cols[1] + C], dv1=g[:, cols[2]:cols[2] + C],
              ld_dq=3 * C, ld_dkv1=3 * C, stride_dkv1_b=L * 3 * C, dkv1_store=True)
    for t, c in zip(f, cols):
        assert torch.equal(g[:, c:c + C], t.to(torch.float16)), c


@pytest.mark.parametrize("M,N,Kd", [(10, 768, 768), (50, 3072, 768), (45, 768, 3072), (128, 200, 96)])
@pytest.mark.parametrize("a_km,b_km", [(1, 1), (1, 0), (0, 0)])
def test_gemm_exact_f32_path(M, N, Kd, a_km, b_km):
    """B f32 selects the exact-f32 MFMA path (decoder query side): fp32-level agreement."""
    k = K()
    if not a_km and M % 4:
        pytest.skip("M-major A needs M % 4 == 0")
    A = torch.randn(M, Kd, device=dev)
    B = torch.randn(N, Kd, device=dev)
    ref = (A.double() @ B.double().t()).float()
    C = torch.empty(M, N, device=dev)
    bias = torch.randn(N, device=dev)
    a_store = A.contiguous() if a_km else A.t().contiguous()
    b_store = B.contiguous() if b_km else B.t().contiguous()
    k.gemm(a_store, b_store, C, M, N, Kd, a_kmajor=bool(a_km), b_kmajor=bool(b_km), flags=16 | 1, bias=bias)
    assert rel(C, ref + bias) < 1e-5
    C2 = torch.zeros(M, N, device=dev)
    k.gemm(a_store, b_store, C2, M, N, Kd, a_kmajor=bool(a_km), b_kmajor=bool(b_km), flags=32 | 1, bias=bias, split_k=3)
    assert rel(C2, ref + bias) < 1e-5


@pytest.mark.parametrize("M,N,R", [(768, 3072, 10), (3072, 768, 50), (768, 768, 64), (3072, 768, 30), (772, 100, 7),
                                   (3076, 776, 9), (36, 68, 9)])
def test_gemm_f32_outer_accumulate(M, N, R):
    """dW (+)= dY^T X, db += colsum(dY) with a skinny reduction (decoder weight gradients): the
    4 x 4 / 2 x 4 per-thread tile kernels, ragged tiles (36 x 68: one partial tile)."""
    k = K()
    dy = torch.randn(R, M, device=dev)
    x = torch.randn(R, N, device=dev)
    dw0 = torch.randn(M, N, device=dev)
    db0 = torch.randn(M, device=dev)
    dw, db = dw0.clone(), db0.clone()
    k.linear_dw(dy, x, dw, bias_grad=db)
    ref = dw0.double() + dy.double().t() @ x.double()
    assert rel(dw, ref.float()) < 1e-5
    assert rel(db, (db0.double() + dy.double().sum(0)).float()) < 1e-5


def test_gemm_f32_splitk_repeatable():
    """The exact-f32 skinny path splits K >= 2048 over workgroups whose partials are handed to the
    last arriver through sc1 stores / loads (gemm_f32.hip).  Re-run it 200 times with a big GEMM on
    another stream (uneven load: arrival order varies) and check every output word each time."""
    k = K()
    M, N, Kd = 10, 768, 3072
    A = torch.randn(M, Kd, device=dev)
    W = torch.randn(N, Kd, device=dev) / math.sqrt(Kd)
    bias = torch.randn(N, device=dev)
    ref = k.linear(A, W, bias, out_f32=True).clone()
    assert rel(ref, (A.double() @ W.double().t() + bias.double()).float()) < 1e-5
    noise = torch.cuda.Stream()
    big = torch.randn(4096, 4096, device=dev)
    bad = 0
    for i in range(200):
        if i % 20 == 0:
            with torch.cuda.stream(noise):
                big = (big @ big).mul_(1e-4)
        y = k.linear(A, W, bias, out_f32=True)
        bad += int(not torch.equal(y, ref))
    torch.cuda.synchronize()
    assert bad == 0


@pytest.mark.parametrize("M", [1, 10, 50])
def test_gemm_f32_skinny_epilogues(M):
    """Decoder query-side linears: GELU + bf16 pre-activation, residual, dGELU on the skinny path."""
    k = K()
    E, FF = 768, 3072
    x = torch.randn(M, E, device=dev)
    w1 = torch.randn(FF, E, device=dev) / math.sqrt(E)
    b1 = torch.randn(FF, device=dev)
    pre = torch.empty(M, FF, device=dev, dtype=torch.bfloat16)
    g = k.linear(x, w1, b1, gelu=True, pre_out=pre, out_f32=True)
    ref_pre = x.double() @ w1.double().t() + b1.double()
    assert rel(pre, ref_pre.float()) < 8e-3
    assert rel(g, F.gelu(ref_pre).float()) < 1e-5
    res = torch.randn(M, E, device=dev)
    w2 = torch.randn(E, FF, device=dev) / math.sqrt(FF)
    y = k.linear(g, w2, None, resid=res, out_f32=True)
    assert rel(y, (g.double() @ w2.double().t() + res.double()).float()) < 1e-5
    dy = torch.randn(M, E, device=dev)
    dgp = k.linear_dx(dy, w2, dgelu_pre=pre)
    pr = pre.double().requires_grad_(True)
    F.gelu(pr).sum().backward()
    assert rel(dgp, ((dy.double() @ w2.double()) * pr.grad).float()) < 1e-5
    dx = k.linear_dx(dgp, w1, resid=res)
    assert rel(dx, (dgp.double() @ w1.double() + res.double()).float()) < 1e-5
    # N = 768 launches split K across workgroups (last arriver reduces in split order): repeated
    # launches — the arrival counters must reset themselves — give bit-identical results
    for _ in range(3):
        assert torch.equal(k.linear_dx(dgp, w1, resid=res), dx)
        assert torch.equal(k.linear(g, w2, None, resid=res, out_f32=True), y)


def test_gemm_epilogues_and_maps():
    k = K()
    M, N, Kd = 520, 256, 160
    x = torch.randn(M, Kd, device=dev)
    w = torch.randn(N, Kd, device=dev) / math.sqrt(Kd)
    b = torch.randn(N, device=dev)
    xb, wb = bf(x), bf(w)
    # GELU + pre-activation store
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    y = k.linear(xb, wb, b, gelu=True, pre_out=pre)
    ref_pre = xb.float() @ wb.float().t() + b
    assert rel(pre, ref_pre) < 1e-2
    assert rel(y, F.gelu(ref_pre)) < 1e-2
    # residual with scatter map + gather map + column scale + row scale
    perm = torch.randperm(M, device=dev).int()
    gat = torch.randperm(M, device=dev).int()
    resid = torch.randn(M, N, device=dev)
    rs = torch.rand(4, device=dev) + 0.5
    out = torch.empty(M, N, device=dev)
    k.linear(xb, wb, b, out=out, resid=resid, c_map=perm, a_map=gat, scale_cols=64, scale_val=0.5,
             row_scale=rs, rows_per_scale=130)
    acc = xb.float()[gat.long()] @ wb.float().t() + b
    acc[:, :64] *= 0.5
    acc = acc * rs[torch.arange(M, device=dev) // 130][:, None]
    ref = resid.clone()
    ref[perm.long()] += acc
    assert rel(out, ref) < 1e-2
    # dX with dgelu and f32 dy with row scale
    dy = torch.randn(M, N, device=dev)
    dx = k.linear_dx(dy, wb, dgelu_pre=None, a_row_scale=rs, a_rows_per_scale=130)
    ref_dx = (bf(dy * rs[torch.arange(M, device=dev) // 130][:, None]).float()) @ wb.float()
    assert rel(dx, ref_dx) < 1e-2
    dz = torch.randn(M, Kd, device=dev)
    dpre = k.linear_dx(bf(dz), bf(w.t().contiguous()), out_f32=False, dgelu_pre=pre)
    pre_r = pre.float().requires_grad_(True)
    F.gelu(pre_r).sum().backward()
    ref_dpre = (bf(dz).float() @ bf(w.t().contiguous()).float()) * pre_r.grad
    assert rel(dpre, ref_dpre) < 2e-2
    # dW with split-K atomics and gathered rows of dy
    dw = torch.zeros(N, Kd, device=dev)
    k.linear_dw(dy, xb, dw, a_map=gat)
    ref_dw = bf(dy[gat.long()]).float().t() @ xb.float()
    assert rel(dw, ref_dw) < 1e-2
    # dW + fused bias gradient (bf16 dY: LDS-DMA kernel, ones-operand MFMA), split-K and not; 9 and 40
    # slices take the slice-parallel reduce (remainder slices included)
    for rows in (M, 4096 + 64, 9 * 1024 + 40, 40 * 1024 + 8):
        dyb = bf(torch.randn(rows, N, device=dev))
        xb2 = bf(torch.randn(rows, Kd, device=dev))
        dw2 = torch.full((N, Kd), 0.25, device=dev)
        db2 = torch.full((N,), 0.5, device=dev)
        k.linear_dw(dyb, xb2, dw2, bias_grad=db2)
        assert rel(dw2, dyb.float().t() @ xb2.float() + 0.25) < 1e-3
        assert rel(db2, dyb.float().sum(0) + 0.5) < 1e-3
    # colsum
    cs = torch.zeros(N, device=dev)
    k.colsum(dy, cs, row_map=gat)
    assert rel(cs, dy.sum(0)) < 1e-4


@pytest.mark.parametrize("R,C", [(3000, 128), (20000, 256), (5000, 1024), (70000, 128)])
def test_layernorm_bwd_param_grads_two_pass(R, C):
    """dw/db through the per-block partials workspace + reduce (block counts of the big Swin LNs)
    against torch and against the atomic fallback."""
    k = K()
    x = torch.randn(R, C, device=dev)
    w = torch.randn(C, device=dev) * 0.2 + 1
    b = torch.randn(C, device=dev) * 0.1
    _, mean, rstd = k.layernorm(x, w, b, 1e-5, out_f32=True)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    dy = torch.randn(R, C, device=dev)
    F.layer_norm(xr, (C,), wr, br, 1e-5).backward(dy)
    outs = []
    for ws in (True, False):
        dx = torch.empty(R, C, device=dev)
        dw = torch.full((C,), 0.5, device=dev)     # accumulates into existing gradients
        db = torch.full((C,), -0.5, device=dev)
        k.layernorm_bwd(dy, x, mean, rstd, w, dx, dw=dw, db=db, workspace=ws)
        assert rel(dx, xr.grad) < 1e-4
        assert rel(dw - 0.5, wr.grad) < 1e-4
        assert rel(db + 0.5, br.grad) < 1e-4
        outs.append((dw, db))
    assert rel(outs[0][0], outs[1][0]) < 1e-5 and rel(outs[0][1], outs[1][1]) < 1e-5


@pytest.mark.parametrize("C,nseg,x_f32", [(128, 1, True), (768, 1, False), (2048, 4, True), (1024, 1, True)])
def test_layernorm_fwd_bwd(C, nseg, x_f32):
    k = K()
    R = 333
    seg = C // nseg
    src = torch.randn(R * nseg, seg, device=dev) * 2 + 0.5
    if not x_f32:
        src = bf(src)
    in_map = torch.randperm(R * nseg, device=dev).int()
    w = torch.randn(C, device=dev) * 0.2 + 1
    b = torch.randn(C, device=dev) * 0.1
    y, mean, rstd = k.layernorm(src, w, b, 1e-5, in_map=in_map, nseg=nseg, rows=R, cols=C, out_f32=True)
    xr = src.float()[in_map.long()].view(R, C).clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (C,), wr, br, 1e-5)
    assert rel(y, yr) < 1e-4
    dy = torch.randn(R, C, device=dev)
    yr.backward(dy)
    dx = torch.zeros(R * nseg, seg, device=dev)
    dres = torch.randn(R * nseg, seg, device=dev)
    dw = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    k.layernorm_bwd(dy, src, mean, rstd, w, dx, in_map=in_map, nseg=nseg, dres=dres, dw=dw, db=db, rows=R, cols=C)
    ref_dx = dres.clone()
    ref_dx[in_map.long()] += xr.grad.view(R * nseg, seg)
    assert rel(dx, ref_dx) < 1e-4
    assert rel(dw, wr.grad) < 1e-4
    assert rel(db, br.grad) < 1e-4
    if nseg == 1:
        # bf16 copy of each LN row's dx, row-scaled (DropPath) and row-permuted (window order)
        sc = torch.rand(7, device=dev) + 0.5
        perm = torch.randperm(R, device=dev).int()
        dx16 = torch.empty(R, C, device=dev, dtype=torch.bfloat16)
        dx2 = torch.zeros(R, C, device=dev)
        k.layernorm_bwd(dy, src, mean, rstd, w, dx2, in_map=in_map, dres=None, rows=R, cols=C, dx16=dx16,
                        dx16_map=perm, dx_scale=sc, dx_scale_rps=50)
        rows_dx = torch.zeros(R, C, device=dev)
        rows_dx = xr.grad * sc[torch.arange(R, device=dev) // 50][:, None]
        ref16 = torch.empty(R, C, device=dev)
        ref16[perm.long()] = rows_dx
        assert rel(dx16, ref16) < 1e-2


def test_scale_cast_bf16():
    k = K()
    x = torch.randn(300, 96, device=dev)
    sc = torch.rand(3, device=dev)
    y = k.scale_cast_bf16(x, sc, 100)
    assert torch.equal(y, bf(x * sc[torch.arange(300, device=dev) // 100][:, None]))


def _wattn_reference(qkv, table, index, region, win_pat, nH, n, c):
    """fp32 reference of video_swin_ori.py:164-186 on the same stored (pre-scaled) q."""
    nw = qkv.shape[0] // n
    C = qkv.shape[1] // 3
    hd = C // nH
    x = qkv.float().view(nw, n, 3, nH, hd).permute(2, 0, 3, 1, 4)
    q = (x[0] / c).requires_grad_(True)
    kk = x[1].clone().requires_grad_(True)
    v = x[2].clone().requires_grad_(True)
    tab = table.clone().requires_grad_(True)
    bias = tab[index[:n, :n].reshape(-1)].view(n, n, nH).permute(2, 0, 1)
    mask = (region[win_pat.long()][:, :, None] != region[win_pat.long()][:, None, :]).float() * -100.0
    s = (q * hd ** -0.5) @ kk.transpose(-1, -2) + bias[None] + mask[:, None]
    o = s.softmax(-1) @ v
    return o.transpose(1, 2).reshape(nw * n, C), (q, kk, v, tab)


@pytest.mark.parametrize("nH,n_win,bias16,gscale", [(4, 9, False, 1.0), (16, 5, False, 1.0), (32, 2, False, 1.0),
                                                   (4, 9, True, 1.0), (16, 5, True, 1.0), (4, 9, True, 1e-12),
                                                   (16, 5, True, 1e6), (3, 4, True, 1.0), (5, 3, False, 1.0)])
def test_window_attention_fwd_bwd(nH, n_win, bias16, gscale):
    """bias16: the backward reads fp16 bias tiles (the Swin-B product path, same rounding as the fused
    forward's); else f32.  gscale: the upstream gradient's magnitude — a batch-mean cross-entropy over
    ~10^5 tokens hands the attention ~1e-6..1e-12-sized gradients; the bias-table bins' fixed point is
    scaled per (window, head), so the relative error must not depend on it.  Odd nH runs the backward's
    one-head-per-workgroup variant (even nH pairs two heads per workgroup)."""
    k = K()
    n, hd = 147, 32
    C = nH * hd
    c = hd ** -0.5 * math.log2(math.e)
    qkv = torch.randn(n_win * n, 3 * C, device=dev)
    qkv[:, :C] *= c
    qkv = bf(qkv)
    table = torch.randn(2535, nH, device=dev)
    index = O.relative_position_index((8, 7, 7)).to(dev)
    n_pat = 3
    region = torch.zeros(n_pat, n, dtype=torch.int32, device=dev)
    region[1, 60:] = 1
    region[2] = torch.randint(0, 3, (n,), device=dev).int()
    win_pat = torch.randint(0, n_pat, (n_win,), device=dev).int()
    bf_ = torch.empty(k.wattn_bias_elems(n_pat, nH), device=dev)
    bb_ = torch.empty_like(bf_)
    k.wattn_bias_build(table, index, n, nH, region, n_pat, bf_, bb_)
    if bias16:
        bb_ = torch.empty(bf_.numel(), device=dev, dtype=torch.float16)
        k.wattn_bias_build(table, index, n, nH, region, n_pat, torch.empty_like(bf_), bb_)
    lse = torch.zeros(n_win, nH, 160, device=dev)
    ref, (q, kk, v, tab) = _wattn_reference(qkv, table, index, region, win_pat, nH, n, c)
    # grouped-by-pattern forward (the product path)
    out = torch.full((n_win * n, C), float("nan"), device=dev, dtype=torch.bfloat16)
    k.wattn_fwd_grouped(qkv, bf_, k.wattn_groups(win_pat, n_win, dev), out, lse, n_win, n, nH)
    assert rel(out, ref) < 1e-2
    out_i = torch.full_like(out, float("nan"))
    lse_i = torch.zeros_like(lse)
    k.wattn_fwd_grouped(qkv, bf_, k.wattn_groups(None, n_win, dev), out_i, lse_i, n_win, n, nH)   # identity grouping
    ref_i, _ = _wattn_reference(qkv, table, index, region, torch.zeros_like(win_pat), nH, n, c)
    assert rel(out_i, ref_i) < 1e-2
    dout = bf(torch.randn(n_win * n, C, device=dev) * gscale)
    ref.backward(dout.float())
    dqkv = torch.full((n_win * n, 3 * C), float("nan"), device=dev, dtype=torch.bfloat16)
    win = (3, 7, 7)
    dbp = torch.full((k.wattn_dbias_part_elems(n_win, nH, win),), float("nan"), device=dev)
    k.wattn_bwd(qkv, out, dout, lse, bb_, win_pat, dqkv, dbp, n_win, n, nH, win)
    tg = torch.zeros(2535, nH, device=dev)   # relative-position bins, summed over windows, -> table rows
    k.wattn_dbias(dbp, n_win, nH, win, k.wattn_bin_rows(index, win), tg)
    # deterministic: a second run gives the same bits
    dqkv2 = torch.empty_like(dqkv)
    tg2 = torch.zeros_like(tg)
    k.wattn_bwd(qkv, out, dout, lse, bb_, win_pat, dqkv2, dbp, n_win, n, nH, win)
    k.wattn_dbias(dbp, n_win, nH, win, k.wattn_bin_rows(index, win), tg2)
    assert torch.equal(dqkv, dqkv2) and torch.equal(tg, tg2)
    d = dqkv.float().view(n_win, n, 3, nH, hd).permute(2, 0, 3, 1, 4)
    assert not torch.isnan(d).any()
    for got, want in ((d[0], q.grad), (d[1], kk.grad), (d[2], v.grad), (tg, tab.grad)):
        assert rel(got, want) < 1.5e-2


@pytest.mark.parametrize("nH,n_win,shifted", [(4, 9, True), (8, 4, False), (16, 5, True), (32, 2, False), (2, 3, True),
                                             (6, 7, True)])
def test_window_attention_fused_qkv_forward(nH, n_win, shifted):
    """lrce_wattn_qkv_fwd (QKV projection + attention in one kernel) vs the two-kernel path (QKV GEMM
    with the q-scale epilogue, then the grouped attention forward) and vs an fp32 reference."""
    k = K()
    n, hd = 147, 32
    C = nH * hd
    c = hd ** -0.5 * math.log2(math.e)
    x = bf(torch.randn(n_win * n, C, device=dev))
    w = bf(torch.randn(3 * C, C, device=dev) / math.sqrt(C))
    bias = torch.randn(3 * C, device=dev) * 0.1
    table = torch.randn(2535, nH, device=dev)
    index = O.relative_position_index((8, 7, 7)).to(dev)
    n_pat = 3 if shifted else 1
    region = torch.zeros(n_pat, n, dtype=torch.int32, device=dev)
    if shifted:
        region[1, 60:] = 1
        region[2] = torch.randint(0, 3, (n,), device=dev).int()
    win_pat = torch.randint(0, n_pat, (n_win,), device=dev).int() if shifted else None
    bf_ = torch.empty(k.wattn_bias_elems(n_pat, nH), device=dev)
    bb_ = torch.empty_like(bf_)
    k.wattn_bias_build(table, index, n, nH, region if shifted else None, n_pat, bf_, bb_)
    bfh = torch.empty(k.wattn_bias_elems(n_pat, nH), device=dev, dtype=torch.float16)   # the fused kernel's fp16 tiles
    k.wattn_bias_build(table, index, n, nH, region if shifted else None, n_pat, bfh, bb_)
    qkv = torch.full((n_win * n, 3 * C), float("nan"), device=dev, dtype=torch.bfloat16)
    out = torch.full((n_win * n, C), float("nan"), device=dev, dtype=torch.bfloat16)
    lse = torch.zeros(n_win, nH, 160, device=dev)
    # windows visited in mask-pattern order (the product path's win_order), or identity
    order = torch.argsort(win_pat.long(), stable=True).int() if shifted else None
    k.wattn_qkv_fwd(x, w, bias, c, bfh, win_pat, qkv, out, lse, n_win, n, nH, win_order=order)
    qkv2 = k.linear(x, w, bias, scale_cols=C, scale_val=c)
    assert rel(qkv, qkv2) < 1e-2                        # same products, bf16 rounding of the outputs
    out2 = torch.empty_like(out)
    lse2 = torch.zeros_like(lse)
    k.wattn_fwd_grouped(qkv2, bf_, k.wattn_groups(win_pat, n_win, dev), out2, lse2, n_win, n, nH)
    assert rel(out, out2) < 1e-2
    assert (lse[..., :n] - lse2[..., :n]).abs().max().item() < 5e-2
    wp = win_pat if shifted else torch.zeros(n_win, dtype=torch.int32, device=dev)
    ref, _ = _wattn_reference(bf(((x.float() @ w.float().t() + bias) * torch.cat(
        [torch.full((C,), c, device=dev), torch.ones(2 * C, device=dev)]))), table, index, region, wp, nH, n, c)
    assert rel(out, ref) < 2e-2


@pytest.mark.parametrize("B,H,Lq,Lk,masked,split,bdiv,drop", [
    (3, 12, 32, 32, True, 0, 1, 0.0), (4, 12, 1, 183, False, 150, 1, 0.0), (2, 12, 40, 40, True, 0, 1, 0.0),
    (10, 12, 1, 191, False, 150, 5, 0.0), (3, 12, 32, 32, True, 0, 1, 0.3), (5, 12, 1, 183, False, 150, 5, 0.5),
    (6, 12, 37, 37, True, 0, 1, 0.1), (45, 12, 40, 40, True, 0, 1, 0.0), (1, 12, 20, 20, False, 0, 1, 0.0)])
def test_mha_fwd_bwd(B, H, Lq, Lk, masked, split, bdiv, drop):
    K().rng_offset(dev).zero_()   # host reference masks assume offset 0
    """Two key segments (video memory shared by `bdiv` rows + text memory), padding mask, dropout."""
    k = K()
    d = 64
    lk1 = split if split else Lk
    lk2 = Lk - lk1
    q = bf(torch.randn(B, Lq, H * d, device=dev))
    kv1 = bf(torch.randn(B // bdiv, lk1, 2 * H * d, device=dev))
    kv2 = bf(torch.randn(B, max(lk2, 1), 2 * H * d, device=dev))
    kmask = torch.ones(B, Lk, dtype=torch.int32, device=dev)
    if masked:
        kmask[0, 20:] = 0
        kmask[-1, 5:] = 0
    out = torch.empty(B, Lq, H * d, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, Lq, device=dev)
    scale = 1 / 8
    desc = k.mha_desc(q, Lq, k1=kv1, v1=kv1[..., H * d:], lk1=lk1, ld_kv1=2 * H * d, stride_kv1_b=lk1 * 2 * H * d,
                      kv1_bdiv=bdiv, k2=kv2 if lk2 else None, v2=kv2[..., H * d:] if lk2 else None, lk2=lk2,
                      ld_kv2=2 * H * d, stride_kv2_b=max(lk2, 1) * 2 * H * d, key_mask=kmask, out=out, lse=lse, B=B, H=H,
                      scale=scale, drop_p=drop, seed=1234)
    k.mha_fwd(desc, out)
    kvf = torch.cat([kv1.float().repeat_interleave(bdiv, 0), kv2.float()[:, :lk2]], 1)
    qr = q.float().view(B, Lq, H, d).transpose(1, 2).requires_grad_(True)
    kr = kvf[..., :H * d].reshape(B, Lk, H, d).transpose(1, 2).contiguous().requires_grad_(True)
    vr = kvf[..., H * d:].reshape(B, Lk, H, d).transpose(1, 2).contiguous().requires_grad_(True)
    s = (qr @ kr.transpose(-1, -2)) * scale + (1 - kmask.float())[:, None, None, :] * -1e30
    P = s.softmax(-1)
    if drop > 0:
        # reproduce the kernel's counter-hash mask on the host: exact recomputation of lrce_uniform
        idx = torch.arange(B * H * Lq * Lk, dtype=torch.int64).view(B, H, Lq, Lk)
        keep = (_hash_uniform(1234, idx) >= drop).to(dev).float() / (1 - drop)
        P = P * keep
    o = (P @ vr).transpose(1, 2).reshape(B, Lq, H * d)
    assert rel(out, o) < 1e-2
    dout = bf(torch.randn(B, Lq, H * d, device=dev))
    o.backward(dout.float())
    dq = torch.empty(B, Lq, H * d, device=dev)
    dkv1 = torch.zeros(B // bdiv, lk1, 2 * H * d, device=dev)
    dkv2 = torch.zeros(B, max(lk2, 1), 2 * H * d, device=dev)
    k.mha_bwd(desc, dout=dout, dq=dq, dk1=dkv1, dv1=dkv1[..., H * d:], ld_dkv1=2 * H * d, stride_dkv1_b=lk1 * 2 * H * d,
              dk2=dkv2 if lk2 else None, dv2=dkv2[..., H * d:] if lk2 else None, ld_dkv2=2 * H * d,
              stride_dkv2_b=max(lk2, 1) * 2 * H * d)
    assert rel(dq, qr.grad.transpose(1, 2).reshape(B, Lq, H * d)) < 1e-2
    gk = kr.grad.transpose(1, 2).reshape(B, Lk, H * d)
    gv = vr.grad.transpose(1, 2).reshape(B, Lk, H * d)
    gk1 = gk[:, :lk1].reshape(B // bdiv, bdiv, lk1, H * d).sum(1)
    gv1 = gv[:, :lk1].reshape(B // bdiv, bdiv, lk1, H * d).sum(1)
    assert rel(dkv1[..., :H * d], gk1) < 1e-2
    assert rel(dkv1[..., H * d:], gv1) < 1e-2
    if lk2:
        assert rel(dkv2[:, :lk2, :H * d], gk[:, lk1:]) < 1e-2
        assert rel(dkv2[:, :lk2, H * d:], gv[:, lk1:]) < 1e-2


def _hash_uniform(seed, idx):
    """Host restatement of lrce_uniform (csrc/common.h): 64-bit mix hash of seed*phi + idx/4, 16 bits
    per index -> [0,1)."""
    import numpy as np
    ix = idx.numpy().astype(np.uint64)
    with np.errstate(over="ignore"):
        v = np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + (ix >> np.uint64(2))
        v ^= v >> np.uint64(33)
        v *= np.uint64(0xff51afd7ed558ccd)
        v ^= v >> np.uint64(33)
        v *= np.uint64(0xc4ceb9fe1a85ec53)
        v ^= v >> np.uint64(33)
    u16 = ((v >> (np.uint64(16) * (ix & np.uint64(3)))) & np.uint64(0xFFFF)).astype(np.float32)
    return torch.from_numpy(u16 * np.float32(1.0 / 65536.0))


def test_dropout_residual_and_groups():
    K().rng_offset(dev).zero_()
    k = K()
    x = torch.randn(4096, device=dev)
    r = torch.randn(4096, device=dev)
    y = k.dropout(x, 0.25, 77, res=r, group=64)
    keep = (_hash_uniform(77, torch.arange(4096) // 64) >= 0.25).to(dev).float()
    assert rel(y, r + x * keep / 0.75) < 1e-6
    dx = k.dropout_bwd(x, 0.25, 77, group=64)
    assert rel(dx, x * keep / 0.75) < 1e-6
    assert 0.6 < keep.mean().item() < 0.9


def test_patch_im2col_matches_conv():
    k = K()
    B, S, T, H, W = 2, 3, 5, 32, 48
    clips = torch.rand(B, S, T, 3, H, W, device=dev)
    Dp = (T + 1) // 2
    patches = torch.empty(B * S * Dp * (H // 4) * (W // 4), 96, device=dev, dtype=torch.bfloat16)
    k.patch_im2col(clips, patches)
    p2 = torch.empty_like(patches)
    k.patch_im2col(O.normalize_clip(clips.cpu()).to(dev).flatten(0, 1).transpose(1, 2).contiguous(), p2, layout='BCTHW', normalize=False)
    assert rel(p2, patches) < 1e-2
    # exact: the same f32 normalisation ((x - mean) * (1 / std), f32 constants) rounded to bf16, zero
    # padded frame, column c*32 + kt*16 + kh*4 + kw of token (clip, d, h, w)
    one = torch.tensor(1.0, device=dev)
    mean = torch.tensor([0.485, 0.456, 0.406], device=dev).view(1, 3, 1, 1, 1)
    istd = (one / torch.tensor([0.229, 0.224, 0.225], device=dev)).view(1, 3, 1, 1, 1)
    x = ((clips.flatten(0, 1).transpose(1, 2) - mean) * istd).to(torch.bfloat16)          # (n, 3, T, H, W)
    x = F.pad(x, (0, 0, 0, 0, 0, T % 2))
    n = B * S
    ref = x.view(n, 3, Dp, 2, H // 4, 4, W // 4, 4).permute(0, 2, 4, 6, 1, 3, 5, 7).reshape(-1, 96)
    assert torch.equal(patches, ref)
    wconv = torch.randn(128, 3, 2, 4, 4, device=dev)
    x = O.normalize_clip(clips.cpu()).to(dev).flatten(0, 1).transpose(1, 2)
    x = F.pad(x, (0, 0, 0, 0, 0, T % 2))
    ref = F.conv3d(x, wconv, stride=(2, 4, 4)).permute(0, 2, 3, 4, 1).reshape(-1, 128)
    got = patches.float() @ wconv.view(128, 96).t()
    assert rel(got, ref) < 1e-2


def test_adamw_matches_torch():
    k = K()
    n = 3 * 1024
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    chunk_tensor = torch.tensor([0, 1, 1], dtype=torch.int32, device=dev)
    lrs = torch.tensor([1e-3, 5e-4], device=dev)
    sumsq = torch.empty(2, device=dev)
    pref = [p[:1024].clone().requires_grad_(True), p[1024:].clone().requires_grad_(True)]
    opt = torch.optim.AdamW([{"params": [pref[0]], "lr": 1e-3}, {"params": [pref[1]], "lr": 5e-4}], betas=(0.9, 0.999))
    reg = 0.001
    for step in range(1, 4):
        k.l2norm_multi(p, chunk_tensor, 3, sumsq, 2)
        pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
        k.adamw_step(p, g, m, v, chunk_tensor, lrs, sumsq, pb, 3, 0.9, 0.999, 1e-8, 0.01, 1.0, reg,
                     1 - 0.9 ** step, 1 - 0.999 ** step)
        opt.zero_grad()
        loss = (pref[0] * g[:1024]).sum() + (pref[1] * g[1024:]).sum() + reg * (pref[0].norm() + pref[1].norm())
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    assert rel(p, torch.cat([pref[0].detach(), pref[1].detach()])) < 1e-5


def test_adamw_keeps_non_finite_gradient_elements_and_scale_backs_off():
    """An element whose gradient is inf / NaN (an overflowed fp16 gradient operand) keeps its parameter
    and moments; the other elements update as usual.  lrce_grad_scale_update halves a scale whose
    recorded max is not finite (the reference's GradScaler backoff) instead of resetting it."""
    k = K()
    n = 2 * 1024
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    g[5], g[1500] = float("inf"), float("nan")
    m, v = torch.full((n,), 0.1, device=dev), torch.full((n,), 0.2, device=dev)
    p0, m0, v0 = p.clone(), m.clone(), v.clone()
    chunk_tensor = torch.tensor([0, 0], dtype=torch.int32, device=dev)
    lrs = torch.tensor([1e-3], device=dev)
    k.adamw_step(p, g, m, v, chunk_tensor, lrs, None, None, 2, 0.9, 0.999, 1e-8, 0.01, 1.0, 0.0, 0.1, 0.001)
    torch.cuda.synchronize()
    for i in (5, 1500):
        assert p[i] == p0[i] and m[i] == m0[i] and v[i] == v0[i]
    ok = torch.ones(n, dtype=torch.bool, device=dev)
    ok[5] = ok[1500] = False
    # (a finite element's update can round to nothing: the bulk must move)
    assert bool(torch.isfinite(p).all()) and (p[ok] != p0[ok]).float().mean().item() > 0.99
    sc = torch.tensor([[64.0, 1 / 64.0, 0.0, 0.0]], device=dev)
    sc.view(torch.int32)[0, 2] = 0x7F800000          # +inf recorded as the max
    k.grad_scale_update(sc)
    torch.cuda.synchronize()
    assert sc[0, 0].item() == 32.0 and sc[0, 1].item() == 1 / 32.0 and sc.view(torch.int32)[0, 2].item() == 0


def test_rng_offset_changes_masks_and_backward_agrees():
    """The device RNG offset (graph replay) moves every mask; dropout backward uses the same mask as
    its forward at the same offset."""
    k = K()
    off = k.rng_offset(dev)
    off.zero_()
    x = torch.randn(1 << 16, device=dev)
    y0 = k.dropout(x, 0.5, 9)
    k.rng_advance(dev)
    y1 = k.dropout(x, 0.5, 9)
    assert not torch.equal(y0 != 0, y1 != 0)
    dx = k.dropout_bwd(torch.ones_like(x), 0.5, 9)
    assert torch.equal(dx != 0, y1 != 0)
    off.zero_()
    assert torch.equal(k.dropout(x, 0.5, 9), y0)


def test_fused_adamw_optimizer_matches_torch_over_steps():
    """FusedAdamW (flat store, device step count, norms carried from the previous update) against
    torch.optim.AdamW + the reference's L2 term (agent_base.py:103-108) on a small module."""
    from lrce.optim import FusedAdamW
    from lrce.runtime import ensure
    torch.manual_seed(3)
    net = torch.nn.Sequential(torch.nn.Linear(24, 40), torch.nn.LayerNorm(40), torch.nn.Linear(40, 8)).to(dev)
    ref = [p.detach().clone().requires_grad_(True) for p in net.parameters()]
    flat = ensure(net)
    groups = [{"params": list(net[0].parameters()), "lr": 2e-3}, {"params": list(net[1:].parameters()), "lr": 1e-3}]
    opt = FusedAdamW(net, groups, lr=1e-3, reg_strength=0.001)
    n0 = len(list(net[0].parameters()))
    topt = torch.optim.AdamW([{"params": ref[:n0], "lr": 2e-3}, {"params": ref[n0:], "lr": 1e-3}])
    for step in range(4):
        gs = [torch.randn_like(r) for r in ref]
        for p, g in zip(net.parameters(), gs):
            flat.g32(p).copy_(g)
        opt.step()
        opt.zero_grad()
        topt.zero_grad()
        loss = sum((r * g).sum() for r, g in zip(ref, gs)) + 0.001 * sum(r.norm() for r in ref)
        loss.backward()
        topt.step()
    for p, r in zip(net.parameters(), ref):
        assert rel(p.detach(), r.detach()) < 1e-5
    assert abs(float(opt.l2_term()) - float(sum(r.norm() for r in ref))) < 1e-3


@pytest.mark.parametrize("M", [10, 45, 100])
def test_fused_dropout_epilogue_matches_separate_launch(M):
    """Decoder linears with the dropout fused into the skinny-GEMM epilogue (M <= 64; M = 100 falls
    back to a dropout launch) give the same bits as GEMM + lrce_dropout / lrce_dropout_bwd."""
    k = K()
    k.rng_offset(dev).zero_()
    E, FF, p = 768, 3072, 0.3
    x = torch.randn(M, E, device=dev)
    w = torch.randn(E, E, device=dev) / math.sqrt(E)
    b = torch.randn(E, device=dev)
    res = torch.randn(M, E, device=dev)
    fused = k.linear(x, w, b, out_f32=True, resid=res, drop=(p, 77, 1))
    ref = k.dropout(k.linear(x, w, b, out_f32=True), p, 77, res=res)
    assert torch.equal(fused, ref)
    head = k.linear(x, w, b, out_f32=True, drop=(p, 78, 64))            # per-head mask (attention-prob dropout)
    assert torch.equal(head, k.dropout(k.linear(x, w, b, out_f32=True), p, 78, group=64))
    w1 = torch.randn(FF, E, device=dev) / math.sqrt(E)
    pre = torch.empty(M, FF, dtype=torch.bfloat16, device=dev)
    g = k.linear(x, w1, None, gelu=True, pre_out=pre, out_f32=True, drop=(p, 79, 1))
    pre2 = torch.empty_like(pre)
    assert torch.equal(g, k.dropout(k.linear(x, w1, None, gelu=True, pre_out=pre2, out_f32=True), p, 79))
    assert torch.equal(pre, pre2)
    dy = torch.randn(M, E, device=dev)
    w2 = torch.randn(E, FF, device=dev) / math.sqrt(FF)
    dg = k.linear_dx(dy, w2, dgelu_pre=pre, drop=(p, 79, 1))
    assert torch.equal(dg, k.dropout_bwd(k.linear_dx(dy, w2, dgelu_pre=pre), p, 79))


@pytest.mark.parametrize("M", [1, 10, 45])
def test_gemm_ln_prologue_forward_and_backward(M):
    """lrce_gemm_ln: the decoder's post-norm LayerNorms folded into the consuming exact-f32 GEMM.
    Mode 1 vs LN then GEMM (f64 torch); mode 2 vs the LN backward + dropout backward then GEMM, with
    the materialised dx / dropped dx and the accumulated gamma / beta gradients."""
    k = K()
    k.rng_offset(dev).zero_()
    E, FF, eps, p = 768, 3072, 1e-12, 0.3
    x = torch.randn(M, E, device=dev) * 3 + 1
    gam = torch.rand(E, device=dev) + 0.5
    bet = torch.randn(E, device=dev)
    w = torch.randn(FF, E, device=dev) / math.sqrt(E)
    b = torch.randn(FF, device=dev)
    mean, rstd, y = torch.empty(M, device=dev), torch.empty(M, device=dev), torch.full((M, E), float("nan"), device=dev)
    pro = k.ln_fwd_prologue(gam, bet, eps, mean=mean, rstd=rstd, y_out=y)
    out = k.linear(x, w, b, out_f32=True, ln=pro)
    xd = x.double()
    ln = F.layer_norm(xd, (E,), gam.double(), bet.double(), eps)
    assert rel(y, ln.float()) < 1e-5
    assert rel(mean, xd.mean(-1).float()) < 1e-5
    assert rel(rstd, (1 / (xd.var(-1, unbiased=False) + eps).sqrt()).float()) < 1e-5
    assert rel(out, (ln @ w.double().t() + b.double()).float()) < 1e-5
    # mode 2: A = dy of the LN output, GEMM consumes dropout_bwd(LN_bwd(dy)) in the dX orientation
    dy = torch.randn(M, E, device=dev)
    w2 = torch.randn(E, FF, device=dev) / math.sqrt(E)    # linear(FF -> E)^T shape [E, FF]: dX = dY' W2
    dgam, dbet = torch.randn(E, device=dev), torch.randn(E, device=dev)
    dg0, db0 = dgam.clone(), dbet.clone()
    dx, dxd = torch.full((M, E), float("nan"), device=dev), torch.full((M, E), float("nan"), device=dev)
    pro = k.ln_bwd_prologue(x, mean, rstd, gam, dgamma=dgam, dbeta=dbet, y_out=dx, y2_out=dxd, drop=(p, 91, 1))
    g = k.linear_dx(dy, w2, ln=pro)
    xr = xd.clone().requires_grad_(True)
    gr, br = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    F.layer_norm(xr, (E,), gr, br, eps).backward(dy.double())
    assert rel(dx, xr.grad.float()) < 1e-5
    assert rel(dgam - dg0, gr.grad.float()) < 1e-5 and rel(dbet - db0, br.grad.float()) < 1e-5
    assert torch.equal(dxd, k.dropout_bwd(dx, p, 91))
    assert rel(g, (dxd.double() @ w2.double()).float()) < 1e-5
    for _ in range(2):   # deterministic (one writer per element)
        dx2 = torch.empty_like(dx)
        g2 = k.linear_dx(dy, w2, ln=k.ln_bwd_prologue(x, mean, rstd, gam, y_out=dx2, drop=(p, 91, 1)))
        assert torch.equal(g2, g) and torch.equal(dx2, dx)


def test_torch_library_ops():
    """torch.ops.lrce.* (lrce/ops.py): the same kernels through the dispatcher, vs fp32 torch."""
    K()
    from lrce import ops  # noqa: F401  (registers the ops)
    torch.manual_seed(3)
    x = bf(torch.randn(300, 256, device=dev))
    w = bf(torch.randn(512, 256, device=dev) / 16)
    b = torch.randn(512, device=dev)
    y = torch.ops.lrce.linear(x, w, b, False, True)
    assert rel(y, x.float() @ w.float().t() + b) < 1e-2
    yg = torch.ops.lrce.linear(x, w, b, True, False)
    assert yg.dtype == torch.bfloat16 and rel(yg, F.gelu(x.float() @ w.float().t() + b)) < 2e-2
    dy = bf(torch.randn(300, 512, device=dev))
    assert rel(torch.ops.lrce.linear_dx(dy, w), dy.float() @ w.float()) < 1e-2
    dw = torch.zeros(512, 256, device=dev)
    torch.ops.lrce.linear_dw_(dw, dy, x)
    assert rel(dw, dy.float().t() @ x.float()) < 1e-2
    xf = torch.randn(300, 256, device=dev)
    g, be = torch.rand(256, device=dev) + 0.5, torch.randn(256, device=dev)
    yl, mean, rstd = torch.ops.lrce.layer_norm(xf, g, be, 1e-5)
    assert rel(yl, F.layer_norm(xf, (256,), g, be, 1e-5)) < 1e-5 and mean.shape == (300,)
    # fused window attention vs the fp32 reference on the same bf16 qkv
    nH, n_win, n = 8, 3, 147
    C = nH * 32
    c = 32 ** -0.5 * math.log2(math.e)
    xw = bf(torch.randn(n_win * n, C, device=dev))
    wq = bf(torch.randn(3 * C, C, device=dev) / math.sqrt(C))
    bq = torch.randn(3 * C, device=dev) * 0.1
    table = torch.randn(2535, nH, device=dev) * 0.1
    index = O.relative_position_index((8, 7, 7)).to(dev)
    region = torch.zeros(2, n, dtype=torch.int32, device=dev)
    region[1, 70:] = 1
    win_pat = torch.tensor([1, 0, 1], dtype=torch.int32, device=dev)
    out, qkv, lse = torch.ops.lrce.window_attention(xw, wq, bq, table, index, n_win, nH, region, win_pat)
    ref, _ = _wattn_reference(qkv, table, index, region, win_pat, nH, n, c)
    assert rel(out, ref) < 2e-2 and lse.shape == (n_win, nH, 160)


def test_torch_library_autograd():
    """Backprop through torch.ops.lrce.window_attention (window_attention_backward: lrce_wattn_bwd +
    lrce_wattn_dbias + the qkv Linear's GEMMs), linear (with GELU) and layer_norm, vs fp32 torch autograd
    of the reference math (video_swin_ori.py:158-189) on the same bf16 values."""
    K()
    from lrce import ops  # noqa: F401
    torch.manual_seed(5)
    nH, n_win, n, hd = 8, 3, 147, 32
    C = nH * hd
    index = O.relative_position_index((8, 7, 7)).to(dev)
    region = torch.zeros(2, n, dtype=torch.int32, device=dev)
    region[1, 70:] = 1
    win_pat = torch.tensor([1, 0, 1], dtype=torch.int32, device=dev)
    xw = bf(torch.randn(n_win * n, C, device=dev)).requires_grad_(True)
    wq = bf(torch.randn(3 * C, C, device=dev) / math.sqrt(C)).requires_grad_(True)
    bq = (torch.randn(3 * C, device=dev) * 0.1).requires_grad_(True)
    table = (torch.randn(2535, nH, device=dev) * 0.3).requires_grad_(True)
    out, qkv, lse = torch.ops.lrce.window_attention(xw, wq, bq, table, index, n_win, nH, region, win_pat)
    gout = torch.randn(out.shape, device=dev)
    (out.float() * gout).sum().backward()
    xr, wr, br, tr = (t.detach().float().requires_grad_(True) for t in (xw, wq, bq, table))
    qkv_r = (xr @ wr.t() + br).view(n_win, n, 3, nH, hd).permute(2, 0, 3, 1, 4)
    bias = tr[index[:n, :n].reshape(-1)].view(n, n, nH).permute(2, 0, 1)
    mask = (region[win_pat.long()][:, :, None] != region[win_pat.long()][:, None, :]).float() * -100.0
    s = (qkv_r[0] * hd ** -0.5) @ qkv_r[1].transpose(-1, -2) + bias[None] + mask[:, None]
    o = (s.softmax(-1) @ qkv_r[2]).transpose(1, 2).reshape(n_win * n, C)
    assert rel(out, o) < 2e-2
    (o * gout).sum().backward()
    for got, ref in ((xw.grad, xr.grad), (wq.grad, wr.grad), (bq.grad, br.grad), (table.grad, tr.grad)):
        assert got is not None and rel(got.float(), ref) < 3e-2, (rel(got.float(), ref), ref.shape)
    # linear (+ GELU) and layer_norm
    x = bf(torch.randn(300, 256, device=dev)).requires_grad_(True)
    w = bf(torch.randn(512, 256, device=dev) / 16).requires_grad_(True)
    b = torch.randn(512, device=dev).requires_grad_(True)
    g = torch.randn(300, 512, device=dev)
    (torch.ops.lrce.linear(x, w, b, True, True) * g).sum().backward()
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    (F.gelu(xr @ wr.t() + br) * g).sum().backward()
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert rel(got.float(), ref) < 2e-2
    xf = torch.randn(300, 256, device=dev, requires_grad=True)
    gm = (torch.rand(256, device=dev) + 0.5).requires_grad_(True)
    be = torch.randn(256, device=dev, requires_grad=True)
    gy = torch.randn(300, 256, device=dev)
    (torch.ops.lrce.layer_norm(xf, gm, be, 1e-5)[0] * gy).sum().backward()
    xr, gr, br = (t.detach().clone().requires_grad_(True) for t in (xf, gm, be))
    (F.layer_norm(xr, (256,), gr, br, 1e-5) * gy).sum().backward()
    for got, ref in ((xf.grad, xr.grad), (gm.grad, gr.grad), (be.grad, br.grad)):
        assert rel(got, ref) < 1e-4


def test_torch_library_patch_embed():
    """torch.ops.lrce.patch_embed (PatchEmbed3D + Normalize, video_swin_ori.py:464-482, video.py:35)
    vs the oracle (conv3d + LayerNorm on the normalized, T-padded clip) and its autograd w.r.t. the
    conv and LayerNorm parameters vs fp32 torch autograd on the same bf16-rounded operands."""
    K()
    from lrce import ops  # noqa: F401
    torch.manual_seed(7)
    B, T, H, W, E = 2, 5, 32, 48, 128
    clips = torch.rand(B, 3, T, H, W, device=dev)
    pw = (torch.randn(E, 3, 2, 4, 4, device=dev) * 0.1).requires_grad_(True)
    pb = (torch.randn(E, device=dev) * 0.1).requires_grad_(True)
    lw = (torch.rand(E, device=dev) + 0.5).requires_grad_(True)
    lb = (torch.randn(E, device=dev) * 0.1).requires_grad_(True)
    x, patches, y, mean, rstd = torch.ops.lrce.patch_embed(clips, pw, pb, lw, lb, True)
    D = (T + 1) // 2
    assert x.shape == (B * D * (H // 4) * (W // 4), E) and patches.dtype == torch.bfloat16
    sd = {"pe.proj.weight": pw.detach().cpu(), "pe.proj.bias": pb.detach().cpu(), "pe.norm.weight": lw.detach().cpu(),
          "pe.norm.bias": lb.detach().cpu()}
    xn = O.normalize_clip(clips.cpu().transpose(1, 2)).transpose(1, 2)
    ref = O.patch_embed(xn, sd, "pe.").reshape(-1, E)
    assert rel(x.cpu(), ref) < 1e-2
    gx = torch.randn(x.shape, device=dev)
    (x * gx).sum().backward()
    # the same math in fp32 on the bf16-rounded im2col operands and weight
    wr, br, lwr, lbr = (t.detach().clone().requires_grad_(True) for t in (pw, pb, lw, lb))
    yr = patches.float() @ wr.reshape(E, 96).to(torch.bfloat16).float().t() + br
    (F.layer_norm(yr, (E,), lwr, lbr, 1e-5) * gx).sum().backward()
    for got, want in ((pw.grad, wr.grad), (pb.grad, br.grad), (lw.grad, lwr.grad), (lb.grad, lbr.grad)):
        assert got is not None and rel(got, want) < 2e-2, (rel(got, want), want.shape)


def test_torch_library_decoder_recurrent():
    """torch.ops.lrce.decoder_recurrent (FusionTransformer.forward, fusionv3.py:27-51: the recurrent
    12-layer decoder over S steps through the native decoder kernels) vs the oracle's
    fusion_transformer on the same weights and memory; text None: FusionVideo (fusionv3.py:70-88)."""
    K()
    from lrce import ops  # noqa: F401
    from lrce.models.fusionv3 import FusionTransformer
    from oracle import weights as W
    torch.manual_seed(9)
    ft = FusionTransformer(768, 0.0)
    sd = W.fill_state_dict({"fusion_model.fusion_transformer." + k: v for k, v in ft.state_dict().items()}, 0)
    ft.load_state_dict({k[len("fusion_model.fusion_transformer."):]: v for k, v in sd.items()})
    params = [p.detach().to(dev) for p in ft.parameters()]
    B, S, L = 3, 2, 21
    video = torch.randn(B, S, 150, 768) * 0.5
    text = torch.randn(B, L, 768) * 0.5
    s = torch.ops.lrce.decoder_recurrent(video.to(dev), text.to(dev), params)
    ref = O.fusion_transformer(video, text, sd).reshape(B, 768)
    assert s.shape == (B, 768) and rel(s.cpu(), ref) < 1e-2, rel(s.cpu(), ref)
    sv = torch.ops.lrce.decoder_recurrent(video.to(dev), None, params)
    refv = O.fusion_video(video, sd).reshape(B, 768)
    assert rel(sv.cpu(), refv) < 1e-2, rel(sv.cpu(), refv)


def test_linear_dw_batched_matches_per_item():
    """lrce_gemm_ptr_batched (a Swin stage's same-shape weight gradients as one launch, one K slice per
    tile) against linear_dw per item (split-K slabs + reduce): dW and the bias gradient to f32 rounding,
    including a K tail (T % 64 != 0) and entries at unrelated addresses."""
    kk = K()
    torch.manual_seed(0)
    T, O, I, n = 1000, 256, 384, 5
    items, ref = [], []
    for j in range(n):
        dy = torch.randn(T, O, device="cuda").to(torch.bfloat16)
        x = torch.randn(T, I, device="cuda").to(torch.bfloat16)
        dw = torch.randn(O, I, device="cuda")
        db = torch.randn(O, device="cuda")
        rw, rb = dw.clone(), db.clone()
        kk.linear_dw(dy, x, rw, bias_grad=rb)
        items.append((dy, x, dw, db))
        ref.append((rw, rb))
    kk.linear_dw_batched(items)
    torch.cuda.synchronize()
    for (dy, x, dw, db), (rw, rb) in zip(items, ref):
        assert rel(dw, rw) < 1e-5 and rel(db, rb) < 1e-5


@pytest.mark.parametrize("n_rep,T,f16,split", [(3, 1000, False, 1), (23, 200, False, 1), (4, 320, True, 1),
                                               (3, 5000, False, 4), (2, 4000, True, 3)])
def test_linear_dw_grouped_mixed_shapes(n_rep, T, f16, split):
    """lrce_gemm_grouped (a Swin stage's linears x blocks as one grid: entries of different shapes, some
    stored (fresh gradients), some accumulated, with and without a bias gradient, C carved from one flat
    buffer like the training layout plus a few separate tensors) against linear_dw per item: dW and db
    to f32 rounding, a K tail (T % 64 != 0), and 92 entries (more than one launch's table) at n_rep 23;
    f16: fp16 operands with a per-entry device alpha (BERT's flush: inverse gradient scales); split: K in
    slices with f32 slabs summed by lrce_slab_sum_grouped (Swin stages 1-2, a K tail in the last slice)."""
    kk = K()
    torch.manual_seed(0)
    shapes = [(256, 384), (128, 256), (384, 128), (512, 512)]
    flat = torch.randn(sum(o * i + o for o, i in shapes) * n_rep + 64, device="cuda")
    off, items, ref = 0, [], []
    for r in range(n_rep):
        for j, (O, I) in enumerate(shapes):
            dt = torch.float16 if f16 else torch.bfloat16
            dy = torch.randn(T, O, device="cuda").to(dt)
            x = torch.randn(T, I, device="cuda").to(dt)
            al = torch.tensor([2.0 ** -(r + j)], device="cuda") if f16 and (r + j) % 3 != 2 else None
            if (r + j) % 5 == 4:
                dw, db = torch.randn(O, I, device="cuda"), torch.randn(O, device="cuda")
            else:
                dw = flat[off:off + O * I].view(O, I); off += O * I
                db = flat[off:off + O]; off += O
            store, bias = (r + j) % 3 == 0, (r + 2 * j) % 4 != 1
            rw, rb = (torch.zeros_like(dw) if store else dw.clone()), db.clone()
            kk.linear_dw(dy, x, rw, bias_grad=rb if bias else None, alpha_dev=al)
            items.append((dy, x, dw, db if bias else None, store, al))
            ref.append((rw, rb))
    kk.linear_dw_grouped(items, split=split)
    torch.cuda.synchronize()
    for (dy, x, dw, db, store, _al), (rw, rb) in zip(items, ref):
        assert rel(dw, rw) < 1e-5
        if db is not None:
            assert rel(db, rb) < 1e-5


@pytest.mark.parametrize("Kd,split,drop", [(768, 3, 0.1), (3072, 4, 0.1), (3072, 4, 0.0)])
def test_linear_resid_ln_matches_unfused(Kd, split, drop):
    """lrce_splitk_reduce_ln after an LRCE_EPI_SLABS split-K GEMM (BERT's output projections: K = 768
    in 3 slices, K = 3072 in 4) against the unfused launches — one GEMM with the bias / dropout / residual
    epilogue, then lrce_layernorm_fwd: same dropout mask, f32 rounding of a different K summation order."""
    kk = K()
    torch.manual_seed(0)
    rows, n = 320, 768
    x = (torch.randn(rows, Kd, device=dev) * 0.5).half()
    w = (torch.randn(n, Kd, device=dev) / Kd ** 0.5).half()
    b = torch.randn(n, device=dev) * 0.1
    resid = torch.randn(rows, n, device=dev)
    gam, bet = 1 + 0.1 * torch.randn(n, device=dev), 0.1 * torch.randn(n, device=dev)
    d = (drop, 12345, 1) if drop > 0 else None
    out16 = torch.empty(rows, n, dtype=torch.float16, device=dev)
    pre, y, mean, rstd = kk.linear_resid_ln(x, w, b, resid, d, gam, bet, 1e-12, split, out16=out16)
    ref_pre = kk.linear(x, w, b, out_f32=True, resid=resid, drop=d)
    ref16 = torch.empty(rows, n, dtype=torch.float16, device=dev)
    ref_y, ref_m, ref_r = kk.layernorm(ref_pre, gam, bet, 1e-12, out_f32=True, bf16_copy=ref16)
    torch.cuda.synchronize()
    assert torch.equal(pre == resid, ref_pre == resid)   # the same dropout mask (a dropped element is resid + 0)
    assert rel(pre, ref_pre) < 1e-5 and rel(y, ref_y) < 1e-4
    assert rel(mean, ref_m) < 1e-4 and rel(rstd, ref_r) < 1e-4
    assert rel(out16.float(), ref16.float()) < 2e-3
