"""The native kernels as PyTorch operators: `torch.ops.lrce.*` (SURVEY §8b's TORCH_LIBRARY surface).

The model's own forward / backward call the C ABI through lrce.kernels directly (its autograd nodes
are whole blocks, see lrce/feature_extractor/video_swin.py and lrce/models/fusionv3.py); these
registrations expose the same kernels to other PyTorch code by name — torch.ops.lrce.linear(...),
torch.compile / FX graphs (each op has a fake implementation for shape propagation), the dispatcher
and profiler — with the C-ABI header (include/lrce_hip.h) unchanged underneath.  Every op runs on a
HIP device only (no CPU kernel is registered: a CPU tensor raises like the rest of the product).
While torch.profiler is recording, every native launch also appears as a `lrce::<entry point>`
range (lrce._native.call).

Ops (reference modules they replace):
  linear(x, w, bias?, gelu, out_f32)              nn.Linear (+ GELU)     video_swin_ori.py:46-57,150,187
  linear_dx(dy, w, out_f32)                       its input gradient
  linear_dw_(dw!, dy, x)                          its weight gradient, accumulated in place
  layer_norm(x, w, b, eps) -> (y, mean, rstd)     nn.LayerNorm           video_swin_ori.py:234,244,319
  window_attention(x, w_qkv, b_qkv, table, index, n_win, nH, region?, win_pat?, window?) -> (out, qkv, lse)
                                                  WindowAttention3D.forward incl. the qkv Linear
                                                  video_swin_ori.py:158-189 (fused kernel)
  window_attention_backward(dout, x, w_qkv, qkv, out, lse, table, index, n_win, nH, region?, win_pat?,
                            window?) -> (dx, dw_qkv, db_qkv, dtable)
                                                  its backward: lrce_wattn_bwd (+ the bias-table
                                                  gradient, lrce_wattn_dbias) and the qkv Linear's
                                                  dX / dW / db GEMMs

  patch_embed(clips, proj_w, proj_b, ln_w, ln_b, normalize) -> (x, patches, y, mean, rstd)
                                                  PatchEmbed3D (+ Normalize)  video_swin_ori.py:464-482,
                                                  video.py:35: im2col -> K = 96 GEMM -> LayerNorm
  decoder_recurrent(video, text, params) -> s     FusionTransformer.forward   fusionv3.py:27-51
                                                  (the recurrent 12-layer decoder over S steps, eval
                                                  mode; text None: FusionVideo, fusionv3.py:70-88)

Autograd (torch.library.register_autograd): linear, layer_norm, window_attention and patch_embed are
differentiable through the same native kernels (linear: dX / dW GEMMs + fused bias gradient;
layer_norm: lrce_layernorm_bwd w.r.t. y; window_attention: window_attention_backward w.r.t. out —
its qkv / lse outputs are saved activations, marked non-differentiable; patch_embed: w.r.t. the conv
and LayerNorm parameters, the clips are data).  decoder_recurrent is a forward (inference) op; the
model's training path differentiates the decoder as one autograd node (lrce/models/fusionv3.py).
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import kernels as K

LOG2E = 1.4426950408889634


@torch.library.custom_op("lrce::linear", mutates_args=())
def linear(x: Tensor, w: Tensor, bias: Optional[Tensor] = None, gelu: bool = False, out_f32: bool = False) -> Tensor:
    """y = x W^T (+ bias) (GELU): bf16 (or f32-A / f32-or-fp16-W skinny) MFMA GEMM, lrce_gemm."""
    return K.linear(x.contiguous(), w.contiguous(), bias, gelu=gelu, out_f32=out_f32)


@linear.register_fake
def _(x, w, bias=None, gelu=False, out_f32=False):
    return x.new_empty((x.shape[0], w.shape[0]), dtype=torch.float32 if out_f32 else x.dtype)


def _linear_setup(ctx, inputs, output):
    x, w, bias, gelu, out_f32 = inputs
    ctx.save_for_backward(x, w, bias)
    ctx.gelu = gelu


def _linear_backward(ctx, dy):
    """dX = dY' W, dW = dY'^T X, db = colsum(dY') with dY' = dY (* GELU'(pre), pre recomputed by the
    same GEMM: the op does not keep its pre-activation)."""
    x, w, bias = ctx.saved_tensors
    dy = dy.contiguous()
    if ctx.gelu:
        pre = K.linear(x.contiguous(), w.contiguous(), bias, out_f32=True)
        t = pre * 0.7071067811865476
        dy = dy.float() * (0.5 * (1.0 + torch.erf(t)) + pre * 0.3989422804014327 * torch.exp(-t * t))
    dyh = dy.to(x.dtype) if x.dtype != torch.float32 else dy
    dx = K.linear_dx(dyh, w.contiguous()).to(x.dtype) if ctx.needs_input_grad[0] else None
    dw = db = None
    if ctx.needs_input_grad[1] or (bias is not None and ctx.needs_input_grad[2]):
        dw = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
        db = torch.zeros(w.shape[0], dtype=torch.float32, device=w.device) if bias is not None else None
        K.linear_dw(dyh, x.contiguous(), dw, bias_grad=db)
        dw = dw.to(w.dtype)
    return dx, dw, db, None, None


linear.register_autograd(_linear_backward, setup_context=_linear_setup)


@torch.library.custom_op("lrce::linear_dx", mutates_args=())
def linear_dx(dy: Tensor, w: Tensor, out_f32: bool = True) -> Tensor:
    """dX = dY W."""
    return K.linear_dx(dy.contiguous(), w.contiguous(), out_f32=out_f32)


@linear_dx.register_fake
def _(dy, w, out_f32=True):
    return dy.new_empty((dy.shape[0], w.shape[1]), dtype=torch.float32 if out_f32 else dy.dtype)


@torch.library.custom_op("lrce::linear_dw_", mutates_args=("dw",))
def linear_dw_(dw: Tensor, dy: Tensor, x: Tensor) -> None:
    """dW += dY^T X (f32 dW, bf16 dY / X; split-K with a deterministic slab reduction)."""
    K.linear_dw(dy.contiguous(), x.contiguous(), dw)


@linear_dw_.register_fake
def _(dw, dy, x):
    return None


@torch.library.custom_op("lrce::layer_norm", mutates_args=())
def layer_norm(x: Tensor, w: Tensor, b: Tensor, eps: float) -> Tuple[Tensor, Tensor, Tensor]:
    """LayerNorm over the last dim of a 2-D f32 / bf16 x: (y f32, mean, rstd)."""
    y, mean, rstd = K.layernorm(x.contiguous(), w, b, eps, out_f32=True)
    return y, mean, rstd


@layer_norm.register_fake
def _(x, w, b, eps):
    rows = x.shape[0]
    return (x.new_empty(x.shape, dtype=torch.float32), x.new_empty((rows,), dtype=torch.float32),
            x.new_empty((rows,), dtype=torch.float32))


def _ln_setup(ctx, inputs, output):
    x, w, b, eps = inputs
    y, mean, rstd = output
    ctx.save_for_backward(x, w, mean, rstd)
    ctx.mark_non_differentiable(mean, rstd)


def _ln_backward(ctx, dy, dmean, drstd):
    """w.r.t. y only (mean / rstd are statistics the backward reuses, not outputs to differentiate)."""
    x, w, mean, rstd = ctx.saved_tensors
    dx = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    dw = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
    db = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
    K.layernorm_bwd(dy.float().contiguous(), x.contiguous(), mean, rstd, w, dx, dw=dw, db=db)
    return dx.to(x.dtype), dw, db, None


layer_norm.register_autograd(_ln_backward, setup_context=_ln_setup)


@torch.library.custom_op("lrce::window_attention", mutates_args=())
def window_attention(x: Tensor, w_qkv: Tensor, b_qkv: Tensor, table: Tensor, index: Tensor, n_win: int, nH: int,
                     region: Optional[Tensor] = None, win_pat: Optional[Tensor] = None,
                     window: Optional[List[int]] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """Fused qkv Linear + 3-D window attention (lrce_wattn_qkv_fwd).  x: bf16 [n_win * n, C] window-
    ordered tokens (LN1 output), w_qkv bf16 [3C, C], b_qkv f32 [3C], table f32 (relative_position_bias_
    table), index int64 (relative_position_index); region int32 [n_pat, n] / win_pat int32 [n_win]:
    the shift mask (None: no shift); window: the (clamped) window shape, (3, 7, 7) by default (n must be
    its volume).  Returns (out bf16 [n_win * n, C] before proj, qkv bf16 (q pre-scaled by
    head_dim^-0.5 * log2(e)), lse f32 [n_win, nH, 160])."""
    C = x.shape[-1]
    n = x.shape[0] // n_win
    n_pat = region.shape[0] if region is not None else 1
    dev = x.device
    bias_f = torch.empty(K.wattn_bias_elems(n_pat, nH), device=dev, dtype=torch.float16)
    bias_b = torch.empty_like(bias_f)
    K.wattn_bias_build(table, index, n, nH, region, n_pat, bias_f, bias_b)
    qkv = torch.empty(x.shape[0], 3 * C, dtype=torch.bfloat16, device=dev)
    out = torch.empty(x.shape[0], C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(n_win, nH, 160, device=dev)
    order = torch.argsort(win_pat.long(), stable=True).to(torch.int32) if win_pat is not None else None
    K.wattn_qkv_fwd(x.contiguous(), w_qkv.contiguous(), b_qkv, (C // nH) ** -0.5 * LOG2E, bias_f, win_pat, qkv, out, lse,
                    n_win, n, nH, win_order=order)
    return out, qkv, lse


@window_attention.register_fake
def _(x, w_qkv, b_qkv, table, index, n_win, nH, region=None, win_pat=None, window=None):
    C = x.shape[-1]
    return (x.new_empty(x.shape, dtype=torch.bfloat16), x.new_empty((x.shape[0], 3 * C), dtype=torch.bfloat16),
            x.new_empty((n_win, nH, 160), dtype=torch.float32))


@torch.library.custom_op("lrce::window_attention_backward", mutates_args=())
def window_attention_backward(dout: Tensor, x: Tensor, w_qkv: Tensor, qkv: Tensor, out: Tensor, lse: Tensor,
                              table: Tensor, index: Tensor, n_win: int, nH: int, region: Optional[Tensor] = None,
                              win_pat: Optional[Tensor] = None,
                              window: Optional[List[int]] = None) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Backward of window_attention w.r.t. its inputs given d(out): lrce_wattn_bwd (one kernel per
    (window, head pair): dQ / dK / dV and the relative-position bins), lrce_wattn_dbias (bins -> table
    rows), then the qkv Linear's dX / dW / db GEMMs.  Returns (dx f32, dw_qkv f32, db_qkv f32, dtable f32)."""
    ws = tuple(window) if window is not None else (3, 7, 7)
    C = x.shape[-1]
    n = x.shape[0] // n_win
    n_pat = region.shape[0] if region is not None else 1
    dev = x.device
    bias_f = torch.empty(K.wattn_bias_elems(n_pat, nH), device=dev, dtype=torch.float16)
    bias_b = torch.empty_like(bias_f)
    K.wattn_bias_build(table, index, n, nH, region, n_pat, bias_f, bias_b)
    dqkv = torch.empty(x.shape[0], 3 * C, dtype=torch.bfloat16, device=dev)
    dbp = torch.empty(K.wattn_dbias_part_elems(n_win, nH, ws), device=dev)
    K.wattn_bwd(qkv, out, dout.to(torch.bfloat16).contiguous(), lse, bias_b, win_pat, dqkv, dbp, n_win, n, nH, ws)
    dtable = torch.zeros(table.shape, dtype=torch.float32, device=dev)
    K.wattn_dbias(dbp, n_win, nH, ws, K.wattn_bin_rows(index, ws), dtable)
    dx = K.linear_dx(dqkv, w_qkv.contiguous())
    dw = torch.zeros(w_qkv.shape, dtype=torch.float32, device=dev)
    db = torch.zeros(3 * C, dtype=torch.float32, device=dev)
    K.linear_dw(dqkv, x.contiguous(), dw, bias_grad=db)
    return dx, dw, db, dtable


@window_attention_backward.register_fake
def _(dout, x, w_qkv, qkv, out, lse, table, index, n_win, nH, region=None, win_pat=None, window=None):
    f = torch.float32
    return (x.new_empty(x.shape, dtype=f), x.new_empty(w_qkv.shape, dtype=f), x.new_empty((w_qkv.shape[0],), dtype=f),
            x.new_empty(table.shape, dtype=f))


def _wattn_setup(ctx, inputs, output):
    x, w_qkv, b_qkv, table, index, n_win, nH, region, win_pat, window = inputs
    out, qkv, lse = output
    ctx.save_for_backward(x, w_qkv, qkv, out, lse, table, index, region, win_pat)
    ctx.n_win, ctx.nH, ctx.window = n_win, nH, window
    ctx.mark_non_differentiable(qkv, lse)


def _wattn_backward(ctx, dout, dqkv, dlse):
    x, w_qkv, qkv, out, lse, table, index, region, win_pat = ctx.saved_tensors
    dx, dw, db, dtable = window_attention_backward(dout, x, w_qkv, qkv, out, lse, table, index, ctx.n_win, ctx.nH,
                                                   region, win_pat, ctx.window)
    return dx.to(x.dtype), dw.to(w_qkv.dtype), db, dtable, None, None, None, None, None, None


window_attention.register_autograd(_wattn_backward, setup_context=_wattn_setup)


@torch.library.custom_op("lrce::patch_embed", mutates_args=())
def patch_embed(clips: Tensor, proj_w: Tensor, proj_b: Tensor, ln_w: Tensor, ln_b: Tensor,
                normalize: bool = False) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """PatchEmbed3D (video_swin_ori.py:464-482): clips (B, 3, T, H, W) f32 (normalize=True applies
    video.py:35's ImageNet Normalize first), T zero-padded to the 2-frame patch, H and W multiples of
    4; conv3d k = s = (2, 4, 4) as im2col (lrce_patch_im2col, bf16 [M, 96]) -> K = 96 GEMM + bias ->
    LayerNorm(E, 1e-5).  Returns (x f32 [B * D' * H' * W', E] channels-last tokens, and the saved
    activations patches bf16 [M, 96], y f32 [M, E] (pre-norm), mean, rstd)."""
    B, C, T, H, W = clips.shape
    if C != 3 or H % 4 or W % 4:
        raise ValueError(f"patch_embed: (B, 3, T, H, W) with H, W multiples of 4, got {tuple(clips.shape)}")
    E = proj_w.shape[0]
    M = B * ((T + 1) // 2) * (H // 4) * (W // 4)
    patches = torch.empty(M, 96, dtype=torch.bfloat16, device=clips.device)
    K.patch_im2col(clips.contiguous(), patches, layout="BCTHW", normalize=normalize)
    w16 = proj_w.reshape(E, 96).to(torch.bfloat16).contiguous()
    y = K.linear(patches, w16, proj_b.float().contiguous(), out_f32=True)
    x, mean, rstd = K.layernorm(y, ln_w.float().contiguous(), ln_b.float().contiguous(), 1e-5, out_f32=True)
    return x, patches, y, mean, rstd


@patch_embed.register_fake
def _(clips, proj_w, proj_b, ln_w, ln_b, normalize=False):
    B, _, T, H, W = clips.shape
    E = proj_w.shape[0]
    M = B * ((T + 1) // 2) * (H // 4) * (W // 4)
    f = torch.float32
    return (clips.new_empty((M, E), dtype=f), clips.new_empty((M, 96), dtype=torch.bfloat16),
            clips.new_empty((M, E), dtype=f), clips.new_empty((M,), dtype=f), clips.new_empty((M,), dtype=f))


def _pe_setup(ctx, inputs, output):
    clips, proj_w, proj_b, ln_w, ln_b, normalize = inputs
    x, patches, y, mean, rstd = output
    ctx.save_for_backward(patches, y, mean, rstd, proj_w, ln_w)
    ctx.mark_non_differentiable(patches, y, mean, rstd)


def _pe_backward(ctx, dx, dpatches, dy_, dmean, drstd):
    """w.r.t. x: the LayerNorm backward writes dy only as the bf16 operand of the conv-weight GEMM,
    whose epilogue sums the bias gradient (as _PatchEmbedFn.backward)."""
    patches, y, mean, rstd, proj_w, ln_w = ctx.saved_tensors
    E = proj_w.shape[0]
    dev = y.device
    dy16 = torch.empty(y.shape, dtype=torch.bfloat16, device=dev)
    dlw = torch.zeros(E, dtype=torch.float32, device=dev)
    dlb = torch.zeros(E, dtype=torch.float32, device=dev)
    K.layernorm_bwd(dx.float().contiguous(), y, mean, rstd, ln_w.float().contiguous(), None, dx16=dy16, dw=dlw, db=dlb)
    dw = torch.zeros(E, 96, dtype=torch.float32, device=dev)
    db = torch.zeros(E, dtype=torch.float32, device=dev)
    K.linear_dw(dy16, patches, dw, bias_grad=db)
    return None, dw.view(proj_w.shape).to(proj_w.dtype), db, dlw, dlb, None


patch_embed.register_autograd(_pe_backward, setup_context=_pe_setup)


_DEC = {}


def _decoder_module(device, n_params):
    """One FusionTransformer per device whose flat store the op's parameters are copied into."""
    m = _DEC.get(device)
    if m is None:
        from .models.fusionv3 import FusionTransformer
        from .runtime import prepare
        m = FusionTransformer(768, 0.0).to(device).eval()
        prepare(m)
        _DEC[device] = m
    if len(list(m.parameters())) != n_params:
        raise ValueError(f"decoder_recurrent: {n_params} parameters given, FusionTransformer has "
                         f"{len(list(m.parameters()))}")
    return m


@torch.library.custom_op("lrce::decoder_recurrent", mutates_args=())
def decoder_recurrent(video: Tensor, text: Optional[Tensor], params: List[Tensor]) -> Tensor:
    """FusionTransformer.forward (fusionv3.py:27-51), eval mode: s <- summarization token; for each of
    the S steps, memory = [video[:, i] (150 tokens); text (L + 1 tokens)], s <- LN(s + Dec12(s,
    memory)) through the native recurrent decoder (csrc/decoder.hip fused attention blocks + the
    exact-f32 FFN GEMMs).  video (B, S, 150, 768) f32, text (B, L + 1, 768) f32 or None (FusionVideo,
    fusionv3.py:70-88); params: FusionTransformer.parameters() in module order (the 12 decoder layers,
    fusion_layer_norm, summarization_token).  Returns s (B, 768) f32."""
    dev = video.device
    m = _decoder_module(dev, len(params))
    from .runtime import ensure
    flat = ensure(m)
    with torch.no_grad():
        for dst, src in zip(m.parameters(), params):
            if dst.shape != src.shape:
                raise ValueError(f"decoder_recurrent: parameter shape {tuple(src.shape)} != {tuple(dst.shape)}")
            dst.copy_(src)
        flat.masters_written()
        B = video.shape[0]
        v = video.contiguous().float()
        v16 = v.to(torch.bfloat16)
        t = text.contiguous().float() if text is not None else None
        t16 = t.to(torch.bfloat16) if t is not None else None
        return m.run(v, v16, t, t16, B, 1).reshape(B, 768).clone()


@decoder_recurrent.register_fake
def _(video, text, params):
    return video.new_empty((video.shape[0], 768), dtype=torch.float32)


def registered() -> List[str]:
    """The lrce operators the dispatcher knows."""
    return ["linear", "linear_dx", "linear_dw_", "layer_norm", "window_attention", "window_attention_backward",
            "patch_embed", "decoder_recurrent"]
