"""LRCE positional embeddings (reference lrce/models/embedding.py) on the gfx950 kernels.

Same parameters (`emb_cls`, `emb_pos`, `emb_len`, `emb_clip`, `layer_norm`), same math:
TextPosEmbed  (embedding.py:17-23): prepend CLS, + positional table, LayerNorm(eps 1e-12).
VideoPosEmbed (embedding.py:47-63): prepend a CLS per (clip, frame-group), + spatial position,
+ frame-group ("len") and + clip embeddings, LayerNorm(eps 1e-12), flatten to 50*groups tokens/clip.
The broadcast adds are one kernel (lrce_video_posembed_fwd / lrce_text_posembed_fwd) feeding the LN
kernel; the caller-side nn.Dropout that follows in the reference (fusionv3.py:156-157,187-188) is
fused here too.
"""
import torch
import torch.nn as nn

from .. import kernels as K

EPS = 1e-12


def init_weight(size):
    """embedding.py:4-7: xavier-normal parameter."""
    w = torch.empty(size)
    nn.init.xavier_normal_(w)
    return nn.Parameter(w, requires_grad=True)


def _g(flat, p):
    return flat.g32(p) if p.requires_grad else None


class TextPosEmbed(nn.Module):
    def __init__(self, seq_len, feature_dim):
        super().__init__()
        self.emb_cls = init_weight((1, 1, feature_dim))
        self.emb_pos = init_weight((1, 1 + seq_len, feature_dim))
        self.layer_norm = nn.LayerNorm(feature_dim, eps=EPS)


class VideoPosEmbed(nn.Module):
    def __init__(self, feature_dim, video_feature_res=(7, 7), frame_sample_size=5, clip_size=6):
        super().__init__()
        self.emb_cls = init_weight((1, 1, 1, 1, feature_dim))
        self.emb_pos = init_weight((1, 1, 1, 1 + video_feature_res[0] * video_feature_res[1], feature_dim))
        self.emb_len = init_weight((1, 1, (frame_sample_size + 1) // 2, 1, feature_dim))
        self.emb_clip = init_weight((1, clip_size, 1, 1, feature_dim))
        self.layer_norm = nn.LayerNorm(feature_dim, eps=EPS)


class VideoEmbedFn(torch.autograd.Function):
    """projection (fusionv3.py:153-154,185) -> VideoPosEmbed -> video_dropout.
    Returns (v f32 (B,S,Tg*50,C), v bf16 copy [non-differentiable])."""

    @staticmethod
    def forward(ctx, vf, proj, pe, flat, p, seed, *params):
        B, S, Tg, P, Cin = vf.shape
        C = pe.layer_norm.weight.shape[0]
        if pe.emb_clip.shape[1] != S:
            raise ValueError(f"emb_clip has {pe.emb_clip.shape[1]} clips but the input has {S} (sum(temporal_scale))")
        dev = vf.device
        rows = B * S * Tg * P
        vf2 = vf.reshape(rows, Cin).contiguous()
        vf16 = torch.empty(rows, Cin, dtype=torch.bfloat16, device=dev)
        K.cast_bf16(vf2, vf16)
        if proj is not None:
            y = K.linear(vf16, flat.w16(proj.weight), proj.bias, out_f32=True)
        else:
            y = vf2
        z = torch.empty(B * S * Tg * (P + 1), C, device=dev)
        K.video_posembed_fwd(y, pe.emb_cls, pe.emb_pos, pe.emb_len, pe.emb_clip, z, B, S, Tg, P, C)
        v, mean, rstd = K.layernorm(z, pe.layer_norm.weight, pe.layer_norm.bias, EPS, out_f32=True)
        v16 = torch.empty(v.shape, dtype=torch.bfloat16, device=dev)
        out = K.dropout(v, p, seed, out_bf16=v16)
        ctx.save = (vf16, z, mean, rstd)
        ctx.proj, ctx.pe, ctx.flat, ctx.p, ctx.seed, ctx.dims = proj, pe, flat, p, seed, (B, S, Tg, P, Cin, C)
        ctx.mark_non_differentiable(v16)
        return out.view(B, S, Tg * (P + 1), C), v16

    @staticmethod
    def backward(ctx, dout, _d16):
        vf16, z, mean, rstd = ctx.save
        proj, pe, flat, p, seed = ctx.proj, ctx.pe, ctx.flat, ctx.p, ctx.seed
        B, S, Tg, P, Cin, C = ctx.dims
        dv = K.dropout_bwd(dout.contiguous().view(-1, C), p, seed) if p > 0 else dout.contiguous().view(-1, C)
        dz = torch.empty_like(z)
        K.layernorm_bwd(dv, z, mean, rstd, pe.layer_norm.weight, dz, dw=_g(flat, pe.layer_norm.weight),
                        db=_g(flat, pe.layer_norm.bias))
        gs = [_g(flat, t) for t in (pe.emb_cls, pe.emb_pos, pe.emb_len, pe.emb_clip)]
        tmp = [g if g is not None else torch.zeros(t.shape, device=dz.device)
               for g, t in zip(gs, (pe.emb_cls, pe.emb_pos, pe.emb_len, pe.emb_clip))]
        if proj is not None:
            # the projection's backward GEMMs read dy as bf16 (LDS-DMA MFMA path), written directly by
            # the positional-embedding backward; the bias gradient rides in the weight-gradient GEMM
            dy16 = torch.empty(B * S * Tg * P, C, dtype=torch.bfloat16, device=dz.device)
            K.video_posembed_bwd(dz, None, tmp[0], tmp[1], tmp[2], tmp[3], B, S, Tg, P, C, dx16=dy16)
            gw, gb = _g(flat, proj.weight), _g(flat, proj.bias)
            if gw is not None:
                K.linear_dw(dy16, vf16, gw, bias_grad=gb)
            elif gb is not None:
                K.colsum(dy16, gb)
            dvf = K.linear_dx(dy16, flat.w16(proj.weight))
        else:
            dvf = torch.empty(B * S * Tg * P, C, device=dz.device)
            K.video_posembed_bwd(dz, dvf, tmp[0], tmp[1], tmp[2], tmp[3], B, S, Tg, P, C)
        ctx.save = None
        flat.notify(list(pe.parameters()) + (list(proj.parameters()) if proj is not None else []))
        return (dvf.view(B, S, Tg, P, Cin),) + (None,) * (5 + len(ctx.needs_input_grad[6:]))


class TextEmbedFn(torch.autograd.Function):
    """TextPosEmbed -> question_dropout.  Returns (t f32 (B,L+1,C), bf16 copy [non-differentiable])."""

    @staticmethod
    def forward(ctx, tf, pe, flat, p, seed, *params):
        B, L, C = tf.shape
        dev = tf.device
        tf2 = tf.contiguous().view(B * L, C)
        z = torch.empty(B * (L + 1), C, device=dev)
        K.text_posembed_fwd(tf2, pe.emb_cls, pe.emb_pos, z, B, L, C)
        t, mean, rstd = K.layernorm(z, pe.layer_norm.weight, pe.layer_norm.bias, EPS, out_f32=True)
        t16 = torch.empty(t.shape, dtype=torch.bfloat16, device=dev)
        out = K.dropout(t, p, seed, out_bf16=t16)
        ctx.save = (z, mean, rstd)
        ctx.pe, ctx.flat, ctx.p, ctx.seed, ctx.dims = pe, flat, p, seed, (B, L, C)
        ctx.mark_non_differentiable(t16)
        return out.view(B, L + 1, C), t16

    @staticmethod
    def backward(ctx, dout, _d16):
        z, mean, rstd = ctx.save
        pe, flat, p, seed = ctx.pe, ctx.flat, ctx.p, ctx.seed
        B, L, C = ctx.dims
        dt = K.dropout_bwd(dout.contiguous().view(-1, C), p, seed) if p > 0 else dout.contiguous().view(-1, C)
        dz = torch.empty_like(z)
        K.layernorm_bwd(dt, z, mean, rstd, pe.layer_norm.weight, dz, dw=_g(flat, pe.layer_norm.weight),
                        db=_g(flat, pe.layer_norm.bias))
        dx = torch.empty(B * L, C, device=dz.device)
        gs = [_g(flat, t) for t in (pe.emb_cls, pe.emb_pos)]
        tmp = [g if g is not None else torch.zeros(t.shape, device=dz.device) for g, t in zip(gs, (pe.emb_cls, pe.emb_pos))]
        K.text_posembed_bwd(dz, dx, tmp[0], tmp[1], B, L, C)
        ctx.save = None
        flat.notify(pe.parameters())
        return (dx.view(B, L, C),) + (None,) * (4 + len(ctx.needs_input_grad[5:]))
