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


class _LayerFn(torch.autograd.Function):
    """One post-norm BERT layer (HF BertLayer): x -> LN(x + drop(attn_out)) -> LN(. + drop(FFN)).

    Forward GEMM / attention operands are IEEE fp16, as under the reference's fp16 autocast
    (agent_oe.py:28; bf16 here would put BERT's rounding error at ~1e-2 of the MC / Count logits).
    Every 16-bit activation the backward needs lives in ONE fp16 buffer, read by the fp16 backward
    as it stands (scaled gradients: backward's docstring)."""

    @staticmethod
    def forward(ctx, x, mask, layer, flat, p, seed, B, L, *params):
        dev = x.device
        rows = B * L
        sa, ao, it, oo = layer.attention.self, layer.attention.output, layer.intermediate, layer.output
        sizes = [rows * HIDDEN] * 6 + [rows * INTER] * 2
        buf = torch.empty(sum(sizes), dtype=torch.float16, device=dev)
        xb, q, k, v, ctxt, h1b, g, pre = _views(buf, rows)
        w = flat.w16h
        K.cast_f16(x, xb)
        _qkv(xb, sa, w, q, k, v, rows)
        lse = torch.empty(B, HEADS, L, device=dev)
        desc = K.mha_desc(q, L, k1=k, v1=v, lk1=L, ld_kv1=HIDDEN, stride_kv1_b=L * HIDDEN, key_mask=mask, out=ctxt,
                          lse=lse, B=B, H=HEADS, scale=0.125, drop_p=p, seed=seed)
        K.mha_fwd(desc, ctxt)
        a = K.linear(ctxt, w(ao.dense.weight), ao.dense.bias, out_f32=True)
        a2 = K.dropout(a, p, seed + 1, res=x)
        h1, m1, r1 = K.layernorm(a2, ao.LayerNorm.weight, ao.LayerNorm.bias, EPS, out_f32=True, bf16_copy=h1b)
        K.linear(h1b, w(it.dense.weight), it.dense.bias, gelu=True, pre_out=pre, out=g)
        o = K.linear(g, w(oo.dense.weight), oo.dense.bias, out_f32=True)
        o2 = K.dropout(o, p, seed + 2, res=h1)
        out, m2, r2 = K.layernorm(o2, oo.LayerNorm.weight, oo.LayerNorm.bias, EPS, out_f32=True)
        ctx.save = (buf, mask, lse, a2, m1, r1, o2, m2, r2)
        ctx.desc = desc
        ctx.layer, ctx.flat, ctx.p, ctx.seed, ctx.B, ctx.L = layer, flat, p, seed, B, L
        return out

    @staticmethod
    def backward(ctx, dout):
        """fp16 backward on scaled gradients, as the reference trains (fp16 autocast + GradScaler,
        agent_oe.py:28,40-42): each f32 residual-stream gradient entering a GEMM gets its own power-of-two
        scale (lrce_grad_scale, on the device), the fp16 operands carry it, and the GEMMs that leave the
        scaled domain (weight gradients, the dX GEMMs with an f32 residual) multiply by 1/S in their
        epilogue.  bf16 here left the top layers' query / key gradients ~0.2 off (near-uniform attention
        rows make them small differences of large terms); fp16 puts them at the reference's own error."""
        buf, mask, lse, a2, m1, r1, o2, m2, r2 = ctx.save
        layer, flat, p, seed, B, L = ctx.layer, ctx.flat, ctx.p, ctx.seed, ctx.B, ctx.L
        sa, ao, it, oo = layer.attention.self, layer.attention.output, layer.intermediate, layer.output
        rows = B * L
        xb, q, k, v, ctxt, h1b, g, pre = _views(buf, rows)   # fp16, as the forward wrote them
        sc = _grad_scales(layer, dout.device)                # (S, 1/S) of the FFN and attention gradients
        inv_f, inv_a = sc[0, 1:2], sc[1, 1:2]
        w = flat.w16h
        dout = dout.contiguous()
        do2 = torch.empty_like(o2)
        K.layernorm_bwd(dout, o2, m2, r2, oo.LayerNorm.weight, do2, dw=_g(flat, oo.LayerNorm.weight),
                        db=_g(flat, oo.LayerNorm.bias))
        K.grad_scale(do2, sc[0])
        do = K.dropout_bwd_f16(do2, p, seed + 2, sc[0])                                   # S_f * d(o)
        _wgrad(flat, oo.dense, do, g, inv_f)
        dh1 = K.linear_dx(do, w(oo.dense.weight), out_f32=False, dgelu_pre=pre)           # S_f * d(pre)
        _wgrad(flat, it.dense, dh1, h1b, inv_f)
        dh1x = K.linear_dx(dh1, w(it.dense.weight), resid=do2, alpha_dev=inv_f)
        da2 = torch.empty_like(a2)
        K.layernorm_bwd(dh1x, a2, m1, r1, ao.LayerNorm.weight, da2, dw=_g(flat, ao.LayerNorm.weight),
                        db=_g(flat, ao.LayerNorm.bias))
        K.grad_scale(da2, sc[1])
        da = K.dropout_bwd_f16(da2, p, seed + 1, sc[1])                                   # S_a * d(a)
        _wgrad(flat, ao.dense, da, ctxt, inv_a)
        dctx = K.linear_dx(da, w(ao.dense.weight), out_f32=False)                         # S_a * d(ctx)
        dqkv = torch.empty(3, rows, HIDDEN, device=dout.device)
        K.mha_bwd(ctx.desc, dout=dctx, dq=dqkv[0], dk1=dqkv[1], dv1=dqkv[2], ld_dkv1=HIDDEN, stride_dkv1_b=L * HIDDEN,
                  dkv1_store=True)
        dqkv16 = torch.empty(3, rows, HIDDEN, dtype=torch.float16, device=dout.device)
        K.cast_f16(dqkv, dqkv16)
        _wgrad_qkv(flat, sa, dqkv16, xb, inv_a, rows)
        dx = K.linear_dx(dqkv16[0], w(sa.query.weight), resid=da2, alpha_dev=inv_a)
        K.linear_dx(dqkv16[1], w(sa.key.weight), out=dx, accumulate=True, alpha_dev=inv_a)
        K.linear_dx(dqkv16[2], w(sa.value.weight), out=dx, accumulate=True, alpha_dev=inv_a)
        ctx.save = ctx.desc = None
        flat.notify(layer.parameters())
        return (dx,) + (None,) * (7 + len(ctx.needs_input_grad[8:]))


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
    if _QKV_BATCHED and sw[0] == sw[1] == sb[0] == sb[1] and sc[0] == sc[1] == rows * HIDDEN and sw[0] != 0:
        if sw[0] > 0:
            K.gemm(xb, ws[0], q, rows, HIDDEN, HIDDEN, flags=N.EPI_BIAS, bias=lins[0].bias, batch=3, stride_b=sw[0],
                   stride_c=sc[0], stride_bias=sb[0], f16=True)
        else:   # the training layout stores parameters in reverse forward order: batch i = value, key, query
            K.gemm(xb, ws[2], v, rows, HIDDEN, HIDDEN, flags=N.EPI_BIAS, bias=lins[2].bias, batch=3, stride_b=-sw[0],
                   stride_c=-sc[0], stride_bias=-sb[0], f16=True)
        return
    for lin, wt, o in zip(lins, ws, (q, k, v)):
        K.linear(xb, wt, lin.bias, out=o)


_QKV_BATCHED = os.environ.get("LRCE_BERT_QKV_BATCHED", "1") != "0"   # A/B knob


def _grad_scales(layer, dev):
    """The layer's two gradient-scale slots [2, 4] f32 (S, 1/S, two arrival words zeroed once: the
    lrce_grad_scale contract), allocated on first use and kept (graph replays reuse them)."""
    sc = getattr(layer, "_lrce_grad_scales", None)
    if sc is None or sc.device != dev:
        sc = torch.zeros(2, 4, device=dev)
        object.__setattr__(layer, "_lrce_grad_scales", sc)
    return sc


def _views(buf, rows):
    """xb, q, k, v, ctxt, h1b [rows, 768] and g, pre [rows, 3072] of one layer's 16-bit buffer."""
    out, o = [], 0
    for cols in (HIDDEN,) * 6 + (INTER,) * 2:
        out.append(buf[o:o + rows * cols].view(rows, cols))
        o += rows * cols
    return out


def _grad16(d32, p, seed):
    """bf16 copy of the dropout-backward of an f32 gradient (the operand of the backward GEMMs)."""
    if p > 0:
        return K.dropout_bwd(d32, p, seed, f32=False)
    out = torch.empty(d32.shape, dtype=torch.bfloat16, device=d32.device)
    K.cast_bf16(d32, out)
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


def _wgrad_qkv(flat, sa, dqkv16, xb, inv_scale, rows):
    """_wgrad of query / key / value as one batched launch when their weight and bias gradients sit at
    one stride in the flat gradient buffer (A/B knob LRCE_BERT_QKV_WGRAD_BATCHED); else three."""
    lins = (sa.query, sa.key, sa.value)
    gws = [_g(flat, l.weight) for l in lins]
    gbs = [_g(flat, l.bias) for l in lins]
    if _QKV_WGRAD_BATCHED and all(t is not None for t in gws + gbs):
        sw = [(gws[i + 1].data_ptr() - gws[i].data_ptr()) // 4 for i in range(2)]
        sb = [(gbs[i + 1].data_ptr() - gbs[i].data_ptr()) // 4 for i in range(2)]
        if sw[0] == sw[1] == sb[0] == sb[1] and sw[0] != 0:
            i0, d = (0, 1) if sw[0] > 0 else (2, -1)     # batch order: ascending gradient addresses
            K.gemm(dqkv16[i0], xb, gws[i0], HIDDEN, HIDDEN, rows, a_kmajor=False, b_kmajor=False, lda=HIDDEN,
                   ldb=HIDDEN, ldc=HIDDEN, flags=N.EPI_ACCUM | N.EPI_BIAS_GRAD, bias=gbs[i0], batch=3,
                   stride_a=d * rows * HIDDEN, stride_c=abs(sw[0]), stride_bias=abs(sb[0]), f16=True,
                   alpha_dev=inv_scale)
            return
    for i, lin in enumerate(lins):
        _wgrad(flat, lin, dqkv16[i], xb, inv_scale)


_QKV_WGRAD_BATCHED = os.environ.get("LRCE_BERT_QKV_WGRAD_BATCHED", "1") != "0"   # A/B knob


class BertModel(nn.Module):
    def __init__(self, n_layers=12, hidden_dropout=0.1, attention_dropout=0.1):
        super().__init__()
        self.embeddings = BertEmbeddings()
        self.encoder = BertEncoder(n_layers)
        self.pooler = BertPooler()
        self.hidden_dropout, self.attention_dropout = hidden_dropout, attention_dropout
        if hidden_dropout != attention_dropout:
            raise ValueError("bert-base uses one dropout rate (0.1) for hidden states and attention probs")

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
        for i, layer in enumerate(self.encoder.layer):
            x = _LayerFn.apply(x, mask, layer, flat, p, seed + 16 * (i + 1), B, L, *layer.parameters())
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
