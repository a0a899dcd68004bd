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
  window_attention(x, w_qkv, b_qkv, table, index, n_win, nH, region?, win_pat?) -> (out, qkv, lse)
                                                  WindowAttention3D.forward incl. the qkv Linear
                                                  video_swin_ori.py:158-189 (fused kernel)
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


@torch.library.custom_op("lrce::window_attention", mutates_args=())
def window_attention(x: Tensor, w_qkv: Tensor, b_qkv: Tensor, table: Tensor, index: Tensor, n_win: int, nH: int,
                     region: Optional[Tensor] = None, win_pat: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """Fused qkv Linear + 3-D window attention (lrce_wattn_qkv_fwd).  x: bf16 [n_win * n, C] window-
    ordered tokens (LN1 output), w_qkv bf16 [3C, C], b_qkv f32 [3C], table f32 (relative_position_bias_
    table), index int64 (relative_position_index); region int32 [n_pat, n] / win_pat int32 [n_win]:
    the shift mask (None: no shift).  Returns (out bf16 [n_win * n, C] before proj, qkv bf16 (q pre-
    scaled by head_dim^-0.5 * log2(e)), lse f32 [n_win, nH, 160])."""
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
def _(x, w_qkv, b_qkv, table, index, n_win, nH, region=None, win_pat=None):
    C = x.shape[-1]
    return (x.new_empty(x.shape, dtype=torch.bfloat16), x.new_empty((x.shape[0], 3 * C), dtype=torch.bfloat16),
            x.new_empty((n_win, nH, 160), dtype=torch.float32))


def registered() -> List[str]:
    """The lrce operators the dispatcher knows."""
    return ["linear", "linear_dx", "linear_dw_", "layer_norm", "window_attention"]
