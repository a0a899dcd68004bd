"""TextExtractor (reference lrce/feature_extractor/text.py:5-17) = BERT-base-uncased encoder on the
gfx950 kernels.

The reference wraps HF `BertModel.from_pretrained('bert-base-uncased')` (transformers 4.20.1) and
returns `last_hidden_state`.  This module re-implements that encoder (published algorithm: word +
position + token-type embeddings -> LN(1e-12) -> 12 post-norm layers of masked 12-head attention
and a GELU(erf) FFN; dropout 0.1 on embeddings, attention probabilities and both residual
branches in train mode) with the SAME parameter names (`bert.embeddings.*`, `bert.encoder.layer.i.*`,
`bert.pooler.dense`), so HF checkpoints load unchanged (`bert.embeddings.position_ids`, a persistent
buffer in 4.20, is accepted and ignored).  The pooler is kept for the schema but, as in the
reference (its output is never used by the loss), not computed.  No network fetch: weights come
from a checkpoint or the caller.  The encoder's forward operands are fp16 (the reference runs
BERT under fp16 autocast), its backward fp16 on scaled gradients (the reference's GradScaler).
"""
import os
import warnings

import torch
import torch.nn as nn

from .. import _native as N
from .. import kernels as K
from ..runtime import ensure

HIDDEN, HEADS, INTER, VOCAB, MAXPOS, TYPES, EPS = 768, 12, 3072, 30522, 512, 2, 1e-12


def _g(flat, p):
    return flat.g32(p) if p.requires_grad else None


class BertEmbeddings(nn.Module):
    def __init__(self):
        super().__init__()
        self.word_embeddings = nn.Embedding(VOCAB, HIDDEN, padding_idx=0)
        self.position_embeddings = nn.Embedding(MAXPOS, HIDDEN)
        self.token_type_embeddings = nn.Embedding(TYPES, HIDDEN)
        self.LayerNorm = nn.LayerNorm(HIDDEN, eps=EPS)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        state_dict.pop(prefix + "position_ids", None)
        state_dict.pop(prefix + "token_type_ids", None)
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)


class BertSelfAttention(nn.Module):
    def __init__(self):
        super().__init__()
        self.query = nn.Linear(HIDDEN, HIDDEN)
        self.key = nn.Linear(HIDDEN, HIDDEN)
        self.value = nn.Linear(HIDDEN, HIDDEN)


class _DenseLN(nn.Module):
    def __init__(self, fan_in):
        super().__init__()
        self.dense = nn.Linear(fan_in, HIDDEN)
        self.LayerNorm = nn.LayerNorm(HIDDEN, eps=EPS)


class BertAttention(nn.Module):
    def __init__(self):
        super().__init__()
        self.self = BertSelfAttention()
        self.output = _DenseLN(HIDDEN)


class BertIntermediate(nn.Module):
    def __init__(self):
        super().__init__()
        self.dense = nn.Linear(HIDDEN, INTER)


class BertLayer(nn.Module):
    def __init__(self):
        super().__init__()
        self.attention = BertAttention()
        self.intermediate = BertIntermediate()
        self.output = _DenseLN(INTER)


class BertEncoder(nn.Module):
    def __init__(self, n_layers=12):
        super().__init__()
        self.layer = nn.ModuleList([BertLayer() for _ in range(n_layers)])


class BertPooler(nn.Module):
    def __init__(self):
        super().__init__()
        self.dense = nn.Linear(HIDDEN, HIDDEN)


# ----------------------------------------------------------------------------------- autograd
class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, types, emb, flat, p, seed, join_token, *params):
        B, L = ids.shape
        rows = B * L
        dev = ids.device
        s = torch.empty(rows, HIDDEN, device=dev)
        K.bert_embed_fwd(ids, types, emb.word_embeddings.weight, emb.position_embeddings.weight,
                         emb.token_type_embeddings.weight, s, rows, L, HIDDEN)
        x, mean, rstd = K.layernorm(s, emb.LayerNorm.weight, emb.LayerNorm.bias, EPS, out_f32=True)
        y = K.dropout(x, p, seed) if p > 0 else x
        ctx.save = (ids, types, s, mean, rstd)
        ctx.emb, ctx.flat, ctx.p, ctx.seed, ctx.L = emb, flat, p, seed, L
        return y

    @staticmethod
    def backward(ctx, dy):
        ids, types, s, mean, rstd = ctx.save
        emb, flat = ctx.emb, ctx.flat
        dy = dy.contiguous()
        dx = K.dropout_bwd(dy, ctx.p, ctx.seed) if ctx.p > 0 else dy
        ds = torch.empty_like(s)
        K.layernorm_bwd(dx, s, mean, rstd, emb.LayerNorm.weight, ds, dw=_g(flat, emb.LayerNorm.weight),
                        db=_g(flat, emb.LayerNorm.bias))
        gw, gp, gt = (_g(flat, emb.word_embeddings.weight), _g(flat, emb.position_embeddings.weight),
                      _g(flat, emb.token_type_embeddings.weight))
        if gw is not None and gp is not None and gt is not None:
            K.bert_embed_bwd(ds, ids, types, gw, gp, gt, s.shape[0], ctx.L, HIDDEN)
        ctx.save = None
        flat.notify(emb.parameters())
        flat.group_done("text")   # every BERT gradient is final: the optimizer may update BERT now
        # join_token (a leaf): its gradient makes autograd join this stream into the caller's at the
        # end of backward (the text branch may run on a side stream, E2EBase.forward)
        dtok = torch.zeros(1, device=dy.device) if ctx.needs_input_grad[6] else None
        return (None,) * 6 + (dtok,) + (None,) * len(ctx.needs_input_grad[7:])


class _Stack:
    """Per-forward state the BERT layers share (one object per BertModel.forward):
    fbuf [n_layers, ...] fp16 — each layer's 16-bit activations (xb, q, k, v, ctxt, h1b, g, pre: the
      forward operands the backward reads), one allocation with a uniform per-layer stride;
    dbuf [n_layers, ...] fp16 — each layer's scaled output gradients (do, dh1, da, dqkv: the dY operands of
      its weight gradients), allocated by the first layer backward;
    scales [n_layers, 2, 4] f32 — the layers' gradient-scale slots (BertModel._grad_scales);
    flush_at — the index of the last layer whose backward runs (the lowest one with a trainable input or
      parameter): its backward issues every layer's weight gradients (_flush_wgrads)."""

    def __init__(self, bert, flat, rows, dev):
        n = len(bert.encoder.layer)
        self.bert, self.flat, self.rows, self.n = bert, flat, rows, n
        self.fbuf = torch.empty(n, rows * _FWD_COLS, dtype=torch.float16, device=dev)
        self.dbuf = None
        self.scales = bert._grad_scales(dev)
        self.flush_at = None
        # delayed gradient scales (lrce_layernorm_bwd_f16s): once a backward has computed every layer's
        # scales from its own maxima, each later step uses the previous step's (the reference's
        # GradScaler likewise keeps one scale across steps); _DELAYED_SCALE = False: per-step scales
        self.delayed = _DELAYED_SCALE and getattr(bert, "_lrce_scales_ready", False)
        self.done = []          # layer indices whose backward has run (their dY in dbuf)
        # the layers' LayerNorm gamma / beta reductions, one batched launch at the flush; a gradient
        # reducer hears of the layers only after that flush
        self.red = K.DeferredGrads()

    def fviews(self, i):
        return _views(self.fbuf[i], self.rows, (HIDDEN,) * 6 + (INTER,) * 2)

    def dviews(self, i):
        if self.dbuf is None:
            self.dbuf = torch.empty(self.n, self.rows * _BWD_COLS, dtype=torch.float16, device=self.fbuf.device)
        return _views(self.dbuf[i], self.rows, (HIDDEN, INTER, HIDDEN, 3 * HIDDEN))


_FWD_COLS = 6 * HIDDEN + 2 * INTER      # xb, q, k, v, ctxt, h1b | g, pre
_BWD_COLS = HIDDEN + INTER + HIDDEN + 3 * HIDDEN   # do, dh1, da, dqkv


class _LayerFn(torch.autograd.Function):
    """One post-norm BERT layer (HF BertLayer): x -> LN(x + drop(attn_out)) -> LN(. + drop(FFN)).

    Forward GEMM / attention operands are IEEE fp16, as under the reference's fp16 autocast
    (agent_oe.py:28; bf16 here would put BERT's rounding error at ~1e-2 of the MC / Count logits).
    Every 16-bit activation the backward needs lives in the layer's slice of the stack's fp16 buffer,
    read by the fp16 backward as it stands (scaled gradients: backward's docstring).  The layer input's
    fp16 copy is written by the previous layer's last LayerNorm; the two residual-branch dropouts ride
    the output-projection GEMMs' epilogues."""

    @staticmethod
    def forward(ctx, x, mask, layer, flat, p, seed, B, L, st, i, *params):
        dev = x.device
        rows = B * L
        sa, ao, it, oo = layer.attention.self, layer.attention.output, layer.intermediate, layer.output
        xb, q, k, v, ctxt, h1b, g, pre = st.fviews(i)
        w = flat.w16h
        if i == 0:
            K.cast_f16(x, xb)
        _qkv(xb, sa, w, q, k, v, rows)
        lse = torch.empty(B, HEADS, L, device=dev)
        desc = K.mha_desc(q, L, k1=k, v1=v, lk1=L, ld_kv1=HIDDEN, stride_kv1_b=L * HIDDEN, key_mask=mask, out=ctxt,
                          lse=lse, B=B, H=HEADS, scale=0.125, drop_p=p, seed=seed)
        K.mha_fwd(desc, ctxt)
        drop1 = (p, seed + 1, 1) if p > 0 else None
        drop2 = (p, seed + 2, 1) if p > 0 else None
        nxt = st.fviews(i + 1)[0] if i + 1 < st.n else None   # the next layer's fp16 input
        # each output projection as split-K slabs + ONE reduce launch that also adds bias, dropout and
        # residual and runs the post-norm LayerNorm (HF BertSelfOutput / BertOutput)
        a2, h1, m1, r1 = K.linear_resid_ln(ctxt, w(ao.dense.weight), ao.dense.bias, x, drop1, ao.LayerNorm.weight,
                                          ao.LayerNorm.bias, EPS, 3, out16=h1b)
        K.linear(h1b, w(it.dense.weight), it.dense.bias, gelu=True, pre_out=pre, out=g)
        o2, out, m2, r2 = K.linear_resid_ln(g, w(oo.dense.weight), oo.dense.bias, h1, drop2, oo.LayerNorm.weight,
                                           oo.LayerNorm.bias, EPS, 4, out16=nxt)
        ctx.save = (mask, lse, a2, m1, r1, o2, m2, r2)
        ctx.desc = desc
        ctx.layer, ctx.flat, ctx.p, ctx.seed, ctx.B, ctx.L, ctx.st, ctx.i = layer, flat, p, seed, B, L, st, i
        return out

    @staticmethod
    def backward(ctx, dout):
        """fp16 backward on scaled gradients, as the reference trains (fp16 autocast + GradScaler,
        agent_oe.py:28,40-42): each f32 residual-stream gradient entering a GEMM gets its own power-of-two
        scale (lrce_grad_scale, on the device), the fp16 operands carry it, and the GEMMs that leave the
        scaled domain (weight gradients, the dX GEMMs with an f32 residual) multiply by 1/S in their
        epilogue.  bf16 here left the top layers' query / key gradients ~0.2 off (near-uniform attention
        rows make them small differences of large terms); fp16 puts them at the reference's own error.
        Weight gradients are deferred: the scaled dY operands stay in the stack's dbuf and the last layer
        backward issues all layers' weight gradients as six batched launches (_flush_wgrads)."""
        mask, lse, a2, m1, r1, o2, m2, r2 = ctx.save
        layer, flat, p, seed, B, L, st, i = ctx.layer, ctx.flat, ctx.p, ctx.seed, ctx.B, ctx.L, ctx.st, ctx.i
        sa, ao, it, oo = layer.attention.self, layer.attention.output, layer.intermediate, layer.output
        rows = B * L
        xb, q, k, v, ctxt, h1b, g, pre = st.fviews(i)      # fp16, as the forward wrote them
        do, dh1, da, dqkv = st.dviews(i)
        sc = st.scales[i]                                   # (S, 1/S) of the FFN and attention gradients
        inv_f, inv_a = sc[0, 1:2], sc[1, 1:2]
        w = flat.w16h
        dout = dout.contiguous()
        do2 = torch.empty_like(o2)
        if i == st.n - 1 and st.delayed:
            K.grad_scale_update(st.scales)      # this step's scales from the last step's maxima
        if st.delayed:   # LN backward + the scaled fp16 operand in one launch (delayed scale)
            K.layernorm_bwd_f16s(dout, o2, m2, r2, oo.LayerNorm.weight, do2, do, sc[0], p, seed + 2,
                                 dw=_g(flat, oo.LayerNorm.weight), db=_g(flat, oo.LayerNorm.bias), defer=st.red)
        else:
            K.layernorm_bwd(dout, o2, m2, r2, oo.LayerNorm.weight, do2, dw=_g(flat, oo.LayerNorm.weight),
                            db=_g(flat, oo.LayerNorm.bias), defer=st.red)
            K.grad_scale(do2, sc[0])
            K.dropout_bwd_f16(do2, p, seed + 2, sc[0], out=do)                            # S_f * d(o)
        K.linear_dx(do, w(oo.dense.weight), out=dh1, out_f32=False, dgelu_pre=pre)        # S_f * d(pre)
        dh1x = _dx_resid(dh1, w(it.dense.weight), do2, inv_f)                          # do2 + (1/S_f) dh1 W1
        da2 = torch.empty_like(a2)
        if st.delayed:
            K.layernorm_bwd_f16s(dh1x, a2, m1, r1, ao.LayerNorm.weight, da2, da, sc[1], p, seed + 1,
                                 dw=_g(flat, ao.LayerNorm.weight), db=_g(flat, ao.LayerNorm.bias), defer=st.red)
        else:
            K.layernorm_bwd(dh1x, a2, m1, r1, ao.LayerNorm.weight, da2, dw=_g(flat, ao.LayerNorm.weight),
                            db=_g(flat, ao.LayerNorm.bias), defer=st.red)
            K.grad_scale(da2, sc[1])
            K.dropout_bwd_f16(da2, p, seed + 1, sc[1], out=da)                            # S_a * d(a)
        dctx = K.linear_dx(da, w(ao.dense.weight), out_f32=False)                         # S_a * d(ctx)
        # dq / dk / dv as fp16 column blocks of ONE [rows, 2304] operand, in the address order of the
        # three weights (so the input gradient is one K = 2304 GEMM when they are contiguous)
        cq, ck, cv = _qkv_cols(sa, w)
        K.mha_bwd(ctx.desc, dout=dctx, dq=dqkv[:, cq:cq + HIDDEN], dk1=dqkv[:, ck:ck + HIDDEN],
                  dv1=dqkv[:, cv:cv + HIDDEN], ld_dq=3 * HIDDEN, ld_dkv1=3 * HIDDEN, stride_dkv1_b=L * 3 * HIDDEN,
                  dkv1_store=True)
        dx = _qkv_dx(dqkv, sa, w, da2, inv_a, rows, (cq, ck, cv))
        ctx.save = ctx.desc = None
        st.done.append(i)
        if i == st.flush_at:
            _flush_wgrads(st)
            st.red.flush(dx)
            for j in st.done:
                flat.notify(st.bert.encoder.layer[j].parameters())
            # a full backward has set every scale: later steps may use delayed scales
            object.__setattr__(st.bert, "_lrce_scales_ready", True)
        return (dx,) + (None,) * (9 + len(ctx.needs_input_grad[10:]))


def _qkv_cols(sa, w):
    """Column offsets of dq, dk, dv in the [rows, 3 * 768] gradient operand: the rank of each weight's
    address among the three (the training layout stores them value, key, query)."""
    ptrs = [w(l.weight).data_ptr() for l in (sa.query, sa.key, sa.value)]
    order = sorted(range(3), key=lambda j: ptrs[j])
    cols = [0, 0, 0]
    for r, j in enumerate(order):
        cols[j] = r * HIDDEN
    return cols


def _qkv_dx(dqkv, sa, w, resid, inv_scale, rows, cols):
    """dX = dq Wq + dk Wk + dv Wv + resid (1/S in the epilogue): ONE K = 2304 GEMM over the stacked
    weights when the three sit back to back in the fp16 shadow, else three accumulating GEMMs."""
    ws = [w(l.weight) for l in (sa.query, sa.key, sa.value)]
    lo = min(ws, key=lambda t: t.data_ptr())
    if sorted(t.data_ptr() - lo.data_ptr() for t in ws) == [0, 2 * HIDDEN * HIDDEN, 4 * HIDDEN * HIDDEN]:
        wstack = torch.as_strided(lo, (3 * HIDDEN, HIDDEN), (HIDDEN, 1))
        return _dx_resid(dqkv, wstack, resid, inv_scale)
    dx = None
    for wt, c in zip(ws, cols):
        a = dqkv[:, c:c + HIDDEN]
        if dx is None:
            dx = K.linear_dx(a, wt, resid=resid, alpha_dev=inv_scale)
        else:
            K.linear_dx(a, wt, out=dx, accumulate=True, alpha_dev=inv_scale)
    return dx


def _dx_resid(dy, w, resid, inv_scale):
    """resid + inv_scale * (dY W) for a deep-K input gradient of the 320-row text branch (K = 2304 /
    3072): split-K slices of 768 (12 K tiles each) write f32 slabs and ONE reduce launch adds them INTO
    resid (an f32 gradient that is dead afterwards: no initialising launch).  A 60-workgroup grid with
    the whole K per workgroup is bound by each workgroup's serial operand intake (36-48 K tiles); the
    slices put 180-240 workgroups on the chip."""
    Kd = w.shape[0]
    split = Kd // 768 if (Kd % 768 == 0 and Kd >= 1536) else 1
    if split == 1:
        return K.linear_dx(dy, w, resid=resid, alpha_dev=inv_scale)
    rows, n = dy.shape[0], w.shape[1]
    ws = torch.empty(split * rows * n, dtype=torch.float32, device=dy.device)
    K.gemm(dy, w, resid, rows, n, Kd, a_kmajor=True, b_kmajor=False, lda=dy.stride(0), ldb=n, ldc=n,
           flags=N.EPI_ATOMIC, split_k=split, workspace=ws, f16=True, alpha_dev=inv_scale)
    return resid


def _qkv(xb, sa, w, q, k, v, rows):
    """query / key / value = xb W^T + b (fp16 out): one batched launch when the three weights and
    biases sit at one stride in the flat buffers and q, k, v at one stride in the layer buffer (3x
    the workgroups of one 320 x 768 x 768 GEMM, 2 launches fewer per layer); else three."""
    lins = (sa.query, sa.key, sa.value)
    ws = [w(l.weight) for l in lins]
    es = 2   # fp16 shadow / q, k, v element size
    sw = [(ws[i + 1].data_ptr() - ws[i].data_ptr()) // es for i in range(2)]
    sb = [(lins[i + 1].bias.data_ptr() - lins[i].bias.data_ptr()) // 4 for i in range(2)]
    sc = [(o2.data_ptr() - o1.data_ptr()) // es for o1, o2 in ((q, k), (k, v))]
    if sw[0] == sw[1] == sb[0] == sb[1] and sc[0] == sc[1] == rows * HIDDEN and sw[0] != 0:
        if sw[0] > 0:
            K.gemm(xb, ws[0], q, rows, HIDDEN, HIDDEN, flags=N.EPI_BIAS, bias=lins[0].bias, batch=3, stride_b=sw[0],
                   stride_c=sc[0], stride_bias=sb[0], f16=True)
        else:   # the training layout stores parameters in reverse forward order: batch i = value, key, query
            K.gemm(xb, ws[2], v, rows, HIDDEN, HIDDEN, flags=N.EPI_BIAS, bias=lins[2].bias, batch=3, stride_b=-sw[0],
                   stride_c=-sc[0], stride_bias=-sb[0], f16=True)
        return
    for lin, wt, o in zip(lins, ws, (q, k, v)):
        K.linear(xb, wt, lin.bias, out=o)


def _views(buf, rows, widths):
    """[rows, width] views of consecutive pieces of a flat 16-bit buffer."""
    out, o = [], 0
    for cols in widths:
        out.append(buf[o:o + rows * cols].view(rows, cols))
        o += rows * cols
    return out


def _wgrad(flat, lin, dy, x16, inv_scale=None):
    """dW += dY^T X with the bias gradient (column sums of dY) fused into the same GEMM; inv_scale (a
    device f32): dY carries a gradient scale, both sums are multiplied by it."""
    gw = _g(flat, lin.weight)
    gb = _g(flat, lin.bias) if lin.bias is not None else None
    if gw is not None:
        K.linear_dw(dy, x16, gw, bias_grad=gb, alpha_dev=inv_scale)
    elif gb is not None:
        if inv_scale is None:
            K.colsum(dy, gb)
        else:   # frozen weight, trainable bias of a scaled gradient (not on the training path)
            t = torch.zeros_like(gb)
            K.colsum(dy, t)
            gb.add_(t * inv_scale)


def _wgrad_items(st, i):
    """The six weight-gradient products of layer i: (linear, dY view, X view, scale slot)."""
    layer = st.bert.encoder.layer[i]
    sa, ao, it, oo = layer.attention.self, layer.attention.output, layer.intermediate, layer.output
    xb, q, k, v, ctxt, h1b, g, pre = st.fviews(i)
    do, dh1, da, dqkv = st.dviews(i)
    cq, ck, cv = _qkv_cols(sa, st.flat.w16h)
    return [(oo.dense, do, g, 0), (it.dense, dh1, h1b, 0), (ao.dense, da, ctxt, 1),
            (sa.query, dqkv[:, cq:cq + HIDDEN], xb, 1), (sa.key, dqkv[:, ck:ck + HIDDEN], xb, 1),
            (sa.value, dqkv[:, cv:cv + HIDDEN], xb, 1)]


def _flush_wgrads(st):
    """Every layer's deferred weight + bias gradients: for each of the six linears ONE batched launch
    over the layers (dW_l += (1/S_l) dY_l^T X_l, db_l += (1/S_l) colsum(dY_l), l = the layers whose
    backward ran), when their gradients, dY / X operands and scale slots sit at uniform strides (the
    flat store lays every layer out alike); else one launch per layer.  48 launches of 60-432
    workgroups on the serial text branch become 6 of 1 000+."""
    flat = st.flat
    layers = sorted(st.done)
    items = {i: _wgrad_items(st, i) for i in layers}
    for j in range(6):
        per = [(i,) + items[i][j] for i in layers]          # (layer, lin, dy, x, slot)
        gws = [_g(flat, lin.weight) for _, lin, _, _, _ in per]
        gbs = [_g(flat, lin.bias) for _, lin, _, _, _ in per]
        if len(per) > 1 and all(t is not None for t in gws + gbs):
            order = sorted(range(len(per)), key=lambda t: gws[t].data_ptr())
            seq = [per[t] for t in order]
            gw, gb = [gws[t] for t in order], [gbs[t] for t in order]

            s_w, s_b = _uniform_stride(gw, 4), _uniform_stride(gb, 4)
            s_a, s_x = _uniform_stride([e[2] for e in seq], 2), _uniform_stride([e[3] for e in seq], 2)
            slots = [st.scales[e[0], e[4], 1:2] for e in seq]
            s_al = _uniform_stride(slots, 4)
            if None not in (s_w, s_b, s_a, s_x, s_al) and s_w > 0 and s_b > 0:
                _, lin, dy, x, _ = seq[0]
                Nn, Kk = lin.weight.shape
                # gradients known to be zero (FlatParams.claim_fresh) are stored, not read-modify-written
                fresh = flat.claim_fresh([q for e in seq for q in (e[1].weight, e[1].bias)]) and _STORE_FRESH
                K.gemm(dy, x, gw[0], Nn, Kk, st.rows, a_kmajor=False, b_kmajor=False, lda=dy.stride(0),
                       ldb=x.stride(0), ldc=Kk, flags=(N.EPI_OUT_F32 if fresh else N.EPI_ACCUM) | N.EPI_BIAS_GRAD,
                       bias=gb[0], batch=len(seq),
                       stride_a=s_a, stride_b=s_x, stride_c=s_w, stride_bias=s_b, f16=True, alpha_dev=slots[0],
                       stride_alpha=s_al)
                continue
        for i, lin, dy, x, slot in per:
            _wgrad(flat, lin, dy, x, st.scales[i, slot, 1:2])


# module switches (tests compare both settings): a batched weight gradient known to start from zero is
# stored, not added (FlatParams.claim_fresh); delayed gradient scales (_Stack.delayed)
_STORE_FRESH = True
_DELAYED_SCALE = True


def _uniform_stride(ts, es):
    """The common address step of consecutive tensors in elements of es bytes (None if not uniform)."""
    ds = {b.data_ptr() - a.data_ptr() for a, b in zip(ts, ts[1:])}
    if len(ds) != 1:
        return None
    d = ds.pop()
    return d // es if d % es == 0 else None


class BertModel(nn.Module):
    def __init__(self, n_layers=12, hidden_dropout=0.1, attention_dropout=0.1):
        super().__init__()
        self.embeddings = BertEmbeddings()
        self.encoder = BertEncoder(n_layers)
        self.pooler = BertPooler()
        self.hidden_dropout, self.attention_dropout = hidden_dropout, attention_dropout
        if hidden_dropout != attention_dropout:
            raise ValueError("bert-base uses one dropout rate (0.1) for hidden states and attention probs")

    def _grad_scales(self, dev):
        """The layers' gradient-scale slots [n_layers, 2, 4] f32 (S, 1/S, two arrival words zeroed once:
        the lrce_grad_scale contract; under delayed scales the last step's max and the found-inf flag),
        allocated on first use and kept (graph replays and the optimizer's overflow guard reuse them)."""
        dev = torch.device(dev)
        if dev.type == "cuda" and dev.index is None:   # "cuda" and "cuda:0" name the same slots
            dev = torch.device("cuda", torch.cuda.current_device())
        sc = getattr(self, "_lrce_grad_scales", None)
        if sc is None or sc.device != dev:
            sc = torch.zeros(len(self.encoder.layer), 2, 4, device=dev)
            object.__setattr__(self, "_lrce_grad_scales", sc)
        return sc

    def lrce_f16_params(self):
        """Parameters whose fp16 shadow the forward reads (the encoder linears; runtime.bind)."""
        return list(self.encoder.parameters())

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, join_token=None):
        flat = ensure(self)
        B, L = input_ids.shape
        dev = input_ids.device
        ids = input_ids.contiguous().to(torch.int64)
        types = (token_type_ids if token_type_ids is not None else torch.zeros_like(ids)).contiguous().to(torch.int64)
        mask = (attention_mask if attention_mask is not None else torch.ones_like(ids)).to(torch.int32).contiguous()
        p = self.hidden_dropout if self.training else 0.0
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
        anchor = [t for t in self.embeddings.parameters()]
        x = _EmbedFn.apply(ids, types, self.embeddings, flat, p, seed, join_token, *anchor)
        st = _Stack(self, flat, B * L, dev)
        for i, layer in enumerate(self.encoder.layer):
            params = list(layer.parameters())
            if st.flush_at is None and torch.is_grad_enabled() and (x.requires_grad or any(q.requires_grad for q in params)):
                st.flush_at = i      # the last layer backward to run issues the deferred weight gradients
            x = _LayerFn.apply(x, mask, layer, flat, p, seed + 16 * (i + 1), B, L, st, i, *params)
        return x.view(B, L, HIDDEN)


BERT_DIR = "./pretrained_models/bert-base-uncased"


def load_bert_weights(bert, path):
    """Load a local bert-base-uncased checkpoint into `bert` (BertModel): a directory holding
    model.safetensors or pytorch_model.bin, or one of those files.  Tensors only (safetensors /
    torch.load(weights_only=True)); HF key prefixes `bert.` and the pretraining heads (`cls.`) are
    handled, TF-era `LayerNorm.gamma/beta` names mapped.  Every encoder / embedding key must be
    present; the pooler may be absent (it is unused by the reference's loss)."""
    if os.path.isdir(path):
        for name in ("model.safetensors", "pytorch_model.bin"):
            if os.path.exists(os.path.join(path, name)):
                path = os.path.join(path, name)
                break
        else:
            raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin under {path}")
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        raw = load_file(path)
    else:
        raw = torch.load(path, map_location="cpu", weights_only=True)
        raw = raw.get("state_dict", raw) if isinstance(raw, dict) else raw
    sd = {}
    for k, v in raw.items():
        if k.startswith("cls.") or not torch.is_tensor(v):
            continue
        k = k[5:] if k.startswith("bert.") else k
        k = k.replace("LayerNorm.gamma", "LayerNorm.weight").replace("LayerNorm.beta", "LayerNorm.bias")
        sd[k] = v
    own = bert.state_dict()
    missing = [k for k in own if k not in sd and not k.startswith("pooler.")]
    if missing:
        raise KeyError(f"BERT checkpoint {path} lacks {len(missing)} keys, e.g. {missing[:3]}")
    bert.load_state_dict({k: v for k, v in sd.items() if k in own or k.endswith("position_ids")}, strict=False)


class TextExtractor(nn.Module):
    """text.py:5-17.  The reference fetches bert-base-uncased by name (text.py:9); this build never
    touches the network: `bert_dir` (a local copy, see load_bert_weights) is loaded when present,
    otherwise the encoder keeps its initialisation with a warning and `pretrained_loaded = False`
    (the training CLI then refuses a non-synthetic run without --allow-random-init).  bert_dir=None:
    random initialisation on purpose (tests, benchmarks)."""

    def __init__(self, bert=None, bert_dir=None):
        super().__init__()
        self.bert = bert if bert is not None else BertModel()
        self.pretrained_loaded = False
        if bert is None and bert_dir:
            if os.path.exists(bert_dir):
                load_bert_weights(self.bert, bert_dir)
                self.pretrained_loaded = True
            else:
                warnings.warn(f"BERT weights {bert_dir} not found: the text encoder keeps its random "
                              "initialisation", stacklevel=2)

    def forward(self, input_ids, attention_mask, token_type_ids, join_token=None):
        return self.bert(input_ids, attention_mask, token_type_ids, join_token=join_token)
