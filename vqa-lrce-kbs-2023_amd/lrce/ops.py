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

Autograd (torch.library.register_autograd): linear, layer_norm and window_attention are
differentiable through the same native kernels (linear: dX / dW GEMMs + fused bias gradient;
layer_norm: lrce_layernorm_bwd w.r.t. y; window_attention: window_attention_backward w.r.t. out —
its qkv / lse outputs are saved activations, marked non-differentiable).
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


def registered() -> List[str]:
    """The lrce operators the dispatcher knows."""
    return ["linear", "linear_dx", "linear_dw_", "layer_norm", "window_attention", "window_attention_backward"]
