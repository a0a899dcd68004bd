"""Video Swin Transformer 3D (Swin-B, patch 2x4x4, window 8x7x7) on the gfx950 kernels.

Re-designed from lrce/feature_extractor/video_swin_ori.py of the reference (a port of the official
Video-Swin-Transformer): same module tree and state-dict keys (`patch_embed.proj/norm`,
`layers.i.blocks.j.{norm1,attn.{relative_position_bias_table,relative_position_index,qkv,proj},
norm2,mlp.{fc1,fc2}}`, `layers.i.downsample.{norm,reduction}`, `norm`), same math, different
execution:

* activations are token-major 2-D tensors, residual stream in f32, GEMM operands in bf16;
* torch.roll + window_partition / window_reverse (video_swin_ori.py:60-88,262,276) are index maps
  (`win2sp`) fused into the LN1 gather and the proj-GEMM scatter epilogue — no copies;
* the relative-position bias + shift mask (:171-179, 346-359) are pre-combined per mask pattern
  into accumulator-order tiles that the fused window-attention kernel starts its MFMA chain from;
* the qkv Linear and the window attention are ONE kernel (csrc/window_fused.hip);
* one autograd Function per block (forward 6 launches, backward 15) with gradients accumulated
  straight into the flat parameter store (lrce/flat.py).
"""

import torch
import torch.nn as nn

from .. import kernels as K
from ..runtime import aux_stream, ensure

LOG2E = 1.4426950408889634


def get_window_size(x_size, window_size, shift_size=None):
    """video_swin_ori.py:91-104: a dim no larger than the window uses the whole dim, zero shift."""
    ws = list(window_size)
    ss = list(shift_size) if shift_size is not None else None
    for i in range(len(x_size)):
        if x_size[i] <= window_size[i]:
            ws[i] = x_size[i]
            if ss is not None:
                ss[i] = 0
    return tuple(ws) if ss is None else (tuple(ws), tuple(ss))


def relative_position_index(window):
    """Pairwise index into the (2Wd-1)(2Wh-1)(2Ww-1) bias table (video_swin_ori.py:133-148)."""
    wd, wh, ww = window
    g = torch.stack(torch.meshgrid(torch.arange(wd), torch.arange(wh), torch.arange(ww), indexing="ij")).flatten(1)
    rel = (g[:, :, None] - g[:, None, :]).permute(1, 2, 0) + torch.tensor([wd - 1, wh - 1, ww - 1])
    return rel[..., 0] * ((2 * wh - 1) * (2 * ww - 1)) + rel[..., 1] * (2 * ww - 1) + rel[..., 2]


# ----------------------------------------------------------------------------------- geometry
class StageGeometry:
    """Index maps for one stage at a given input size (cached per device).

    Windows tile the volume padded up to whole windows (video_swin_ori.py:253-258 pads norm1's output
    with zeros, :346 builds the mask over the padded volume): the window-order maps run over the
    padded volume and mark padded positions -1 (the LN1 gather writes zero rows there, the proj GEMM
    drops them, the LN1 backward skips them).  Spatial tensors keep the unpadded M rows; window-order
    tensors (LN1 output, qkv, attention output) have M_win = n_win * n rows."""

    def __init__(self, nc, D, H, W, window, device):
        half = tuple(i // 2 for i in window)
        ws, ss = get_window_size((D, H, W), window, half)
        self.nc, self.D, self.H, self.W = nc, D, H, W
        self.ws, self.ss = ws, ss
        self.Dp, self.Hp, self.Wp = (-(-D // ws[0]) * ws[0], -(-H // ws[1]) * ws[1], -(-W // ws[2]) * ws[2])
        self.padded = (self.Dp, self.Hp, self.Wp) != (D, H, W)
        self.n = ws[0] * ws[1] * ws[2]
        self.nW = (self.Dp // ws[0]) * (self.Hp // ws[1]) * (self.Wp // ws[2])
        self.n_win = nc * self.nW
        self.M = nc * D * H * W
        self.M_win = self.n_win * self.n
        self.rows_per_clip = D * H * W
        self.win_rows_per_clip = self.nW * self.n
        self.win2sp = self._win_map((0, 0, 0), device)
        self.sp2win = self._inverse(self.win2sp)
        self.shifted = any(s > 0 for s in ss)
        if self.shifted:
            self.win2sp_shift = self._win_map(ss, device)
            self.sp2win_shift = self._inverse(self.win2sp_shift)
            self.region, self.win_pat, self.n_pat = self._mask_patterns(device)
            self.groups_shift = K.wattn_groups(self.win_pat, self.n_win, device)
            # the fused forward visits windows grouped by mask pattern (stable): the workgroups one XCD
            # runs then share few patterns' bias tiles in its L2
            self.win_order = torch.argsort(self.win_pat.long(), stable=True).to(torch.int32).contiguous()
        self.groups = K.wattn_groups(None, self.n_win, device)
        # PatchMerging pads odd H / W with zeros before its 2x2 gather (video_swin_ori.py:328-331)
        self.Hm, self.Wm = -(-H // 2), -(-W // 2)
        self.M_merged = nc * D * self.Hm * self.Wm
        self.merge_map = self._merge_map(device)

    def _win_map(self, shift, device):
        D, H, W = self.D, self.H, self.W
        Dp, Hp, Wp = self.Dp, self.Hp, self.Wp
        wd, wh, ww = self.ws
        ar = lambda n: torch.arange(n, device=device)
        b, iwd, iwh, iww, td, th, tw = torch.meshgrid(ar(self.nc), ar(Dp // wd), ar(Hp // wh), ar(Wp // ww), ar(wd),
                                                      ar(wh), ar(ww), indexing="ij")
        d = (iwd * wd + td + shift[0]) % Dp
        h = (iwh * wh + th + shift[1]) % Hp
        w = (iww * ww + tw + shift[2]) % Wp
        row = ((b * D + d) * H + h) * W + w
        row = torch.where((d < D) & (h < H) & (w < W), row, torch.full_like(row, -1))
        return row.reshape(-1).to(torch.int32).contiguous()

    def _inverse(self, perm):
        """spatial row -> window-order row (every real token sits in exactly one window)"""
        inv = torch.empty(self.M, dtype=perm.dtype, device=perm.device)
        live = perm >= 0
        inv[perm[live].long()] = torch.arange(perm.numel(), device=perm.device, dtype=perm.dtype)[live]
        return inv

    def _mask_patterns(self, device):
        """Region labels of compute_mask (video_swin_ori.py:346-359) over the padded, rolled volume,
        as per-window region-id rows, de-duplicated into patterns (windows away from the rolled
        border all share the all-zero pattern)."""
        D, H, W = self.Dp, self.Hp, self.Wp
        ws, ss = self.ws, self.ss
        lab = torch.zeros(D, H, W, dtype=torch.int32)
        cnt = 0
        for sd in (slice(-ws[0]), slice(-ws[0], -ss[0]), slice(-ss[0], None)):
            for sh in (slice(-ws[1]), slice(-ws[1], -ss[1]), slice(-ss[1], None)):
                for sw in (slice(-ws[2]), slice(-ws[2], -ss[2]), slice(-ss[2], None)):
                    lab[sd, sh, sw] = cnt
                    cnt += 1
        wd, wh, ww = ws
        win = lab.view(D // wd, wd, H // wh, wh, W // ww, ww).permute(0, 2, 4, 1, 3, 5).reshape(-1, self.n)
        patterns, inv = torch.unique(win, dim=0, return_inverse=True)
        win_pat = inv.to(torch.int32).repeat(self.nc)
        return patterns.to(torch.int32).contiguous().to(device), win_pat.contiguous().to(device), patterns.shape[0]

    def _merge_map(self, device):
        """PatchMerging concat order x0..x3 = (h,w) offsets (0,0),(1,0),(0,1),(1,1) (:333-337); sources
        past an odd H / W are the zero padding (-1)."""
        nc, D, H, W = self.nc, self.D, self.H, self.W
        ar = lambda n: torch.arange(n, device=device)
        b, d, i, j, s = torch.meshgrid(ar(nc), ar(D), ar(self.Hm), ar(self.Wm), ar(4), indexing="ij")
        h = 2 * i + torch.tensor([0, 1, 0, 1], device=device)[s]
        w = 2 * j + torch.tensor([0, 0, 1, 1], device=device)[s]
        row = ((b * D + d) * H + h) * W + w
        row = torch.where((h < H) & (w < W), row, torch.full_like(row, -1))
        return row.reshape(-1).to(torch.int32).contiguous()


_GEO_CACHE = {}


def stage_geometry(nc, D, H, W, window, device):
    key = (nc, D, H, W, tuple(window), str(device))
    g = _GEO_CACHE.get(key)
    if g is None:
        if len(_GEO_CACHE) > 64:
            _GEO_CACHE.clear()
        g = _GEO_CACHE[key] = StageGeometry(nc, D, H, W, window, device)
    return g


def _g(flat, p):
    return flat.g32(p) if p.requires_grad else None


# ----------------------------------------------------------------------------------- modules
class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden_features, in_features)


class WindowAttention3D(nn.Module):
    def __init__(self, dim, window_size, num_heads):
        super().__init__()
        self.dim, self.window_size, self.num_heads = dim, window_size, num_heads
        wd, wh, ww = window_size
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * wd - 1) * (2 * wh - 1) * (2 * ww - 1), num_heads))
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)
        self.register_buffer("relative_position_index", relative_position_index(window_size))
        self.qkv = nn.Linear(dim, 3 * dim)
        self.proj = nn.Linear(dim, dim)


class SwinTransformerBlock3D(nn.Module):
    def __init__(self, dim, num_heads, window_size, shift_size, drop_path=0.0):
        super().__init__()
        self.dim, self.num_heads, self.window_size, self.shift_size = dim, num_heads, window_size, shift_size
        self.drop_path = drop_path
        self.norm1 = nn.LayerNorm(dim)
        self.attn = WindowAttention3D(dim, window_size, num_heads)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = Mlp(dim, 4 * dim)

    def tensors(self):
        return [p for p in self.parameters()]


class PatchMerging(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = nn.LayerNorm(4 * dim)


class BasicLayer(nn.Module):
    def __init__(self, dim, depth, num_heads, window_size, drop_path, downsample):
        super().__init__()
        self.window_size = window_size
        self.shift_size = tuple(i // 2 for i in window_size)
        self.blocks = nn.ModuleList([
            SwinTransformerBlock3D(dim, num_heads, window_size, (0, 0, 0) if i % 2 == 0 else self.shift_size,
                                   drop_path[i]) for i in range(depth)])
        self.downsample = PatchMerging(dim) if downsample else None


class PatchEmbed3D(nn.Module):
    def __init__(self, patch_size=(2, 4, 4), in_chans=3, embed_dim=128):
        super().__init__()
        self.patch_size, self.embed_dim = patch_size, embed_dim
        self.proj = nn.Conv3d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = nn.LayerNorm(embed_dim)


# ----------------------------------------------------------------------------------- autograd
class _PatchEmbedFn(torch.autograd.Function):
    """im2col(+normalize, +T pad) -> K=96 GEMM (+bias) -> LN(128); video_swin_ori.py:464-482."""

    @staticmethod
    def forward(ctx, clips, pe, flat, layout, normalize, *params):
        if layout == "BSTCHW":
            B, S, T, _, H, W = clips.shape
            nc = B * S
        else:
            B, _, T, H, W = clips.shape
            nc = B
        if H % 4 or W % 4:
            # the reference zero-pads H / W up to the 4x4 patch (video_swin_ori.py:466-470); the fused
            # im2col reads whole patches only
            raise ValueError(f"PatchEmbed3D: frame size {H}x{W} is not a multiple of the 4x4 patch (unsupported)")
        clips = clips.contiguous()
        Dp, Hp, Wp = (T + 1) // 2, H // 4, W // 4
        M = nc * Dp * Hp * Wp
        patches = torch.empty(M, 96, dtype=torch.bfloat16, device=clips.device)
        K.patch_im2col(clips, patches, layout=layout, normalize=normalize)
        w16 = flat.w16(pe.proj.weight).view(pe.embed_dim, 96)
        y = K.linear(patches, w16, pe.proj.bias, out_f32=True)
        x, mean, rstd = K.layernorm(y, pe.norm.weight, pe.norm.bias, 1e-5, out_f32=True)
        ctx.pe, ctx.flat = pe, flat
        ctx.patches, ctx.y, ctx.mean, ctx.rstd = patches, y, mean, rstd
        ctx.shape = (nc, Dp, Hp, Wp)
        return x

    @staticmethod
    def backward(ctx, dx):
        pe, flat = ctx.pe, ctx.flat
        # the LN backward writes dy only as the bf16 operand of the conv-weight gradient GEMM, whose
        # epilogue also sums the bias gradient (no f32 dy round trip, no separate column sum)
        dy16 = torch.empty(ctx.y.shape, dtype=torch.bfloat16, device=dx.device)
        K.layernorm_bwd(dx.contiguous(), ctx.y, ctx.mean, ctx.rstd, pe.norm.weight, None, dx16=dy16,
                        dw=_g(flat, pe.norm.weight), db=_g(flat, pe.norm.bias))
        gw, gb = _g(flat, pe.proj.weight), _g(flat, pe.proj.bias)
        if gw is not None:
            K.linear_dw(dy16, ctx.patches, gw.view(pe.embed_dim, 96), bias_grad=gb)
        elif gb is not None:
            K.colsum(dy16, gb)
        flat.notify(pe.parameters())
        return (None,) * (5 + len(list(pe.parameters())))


# LayerNorm-backward input gradients of rows this wide or wider stay f32 (the LN backward's bf16 loads
# measured slower there, tools/ln_bench.py)
_LN_F32_WIDE = 1024


def _drop_path_scale(rate, nc, device, training):
    """timm DropPath (video_swin_ori.py:243,299): per-sample keep mask / keep_prob, here per clip."""
    if not training or rate <= 0.0:
        return None
    keep = 1.0 - rate
    return torch.floor(keep + torch.rand(nc, device=device)) / keep


_KEEP_CACHE = {}


def _drop_path_scales(swin, nc, device):
    """Both DropPath scale vectors of every block of one forward, drawn in ONE batch (4 launches per
    step instead of 4 per DropPath): [(dp1, dp2) per block] or None in eval mode.  Blocks whose rate
    is 0 (the first, linspace(0, 0.2, 24)[0]) get None, as in _drop_path_scale."""
    if not swin.training:
        return None
    rates = [blk.drop_path for layer in swin.layers for blk in layer.blocks]
    key = (tuple(rates), str(device))
    keep = _KEEP_CACHE.get(key)
    if keep is None:
        keep = _KEEP_CACHE[key] = torch.tensor([[1.0 - r] for r in rates for _ in range(2)], device=device)
    s = torch.floor(keep + torch.rand(len(rates) * 2, nc, device=device)) / keep
    return [(s[2 * i], s[2 * i + 1]) if r > 0.0 else (None, None) for i, r in enumerate(rates)]


def _wgrad(flat, lin, dy16, x16, defer=None):
    """dW += dY^T X and db += colsum(dY) in one GEMM launch (bias sum fused via LRCE_EPI_BIAS_GRAD);
    defer: a DeferredGrads whose flush issues the stage's same-shape weight gradients as one batched
    launch (no split-K slabs / reduce) — the operands stay alive until then."""
    gw = _g(flat, lin.weight)
    gb = _g(flat, lin.bias) if lin.bias is not None else None
    if gw is not None:
        if (defer is not None and _DEFER_WGRAD and dy16.dtype == torch.bfloat16 and x16.dtype == torch.bfloat16
                and defer.wants_dw(gw.shape[0], gw.shape[1], x16.shape[0])):
            ps = [lin.weight] + ([lin.bias] if gb is not None else [])
            defer.dw.append((dy16, x16, gw, gb, flat.claim_fresh(ps) and _STORE_FRESH))
        else:
            K.linear_dw(dy16, x16, gw, bias_grad=gb)
    elif gb is not None:
        K.colsum(dy16, gb)


def _bin_rows(at, window):
    """Bias-gradient bin -> table row map of one attention module, cached against its index buffer."""
    idx = at.relative_position_index
    key = (idx.data_ptr(), idx._version, tuple(window), idx.device)
    hit = getattr(at, "_lrce_bin_rows", None)
    if hit is None or hit[0] != key:
        hit = (key, K.wattn_bin_rows(idx, window))
        object.__setattr__(at, "_lrce_bin_rows", hit)
    return hit[1]


_HANDOFF = True   # tests switch it off to compare against the separate scale-cast launch


class _Handoff:
    """Backward link between two consecutive blocks of a stage.  The later block's LN1 backward (which
    writes dx, the earlier block's output gradient) also writes it as bf16 scaled by the earlier
    block's DropPath dp2 — the A operand of that block's MLP GEMMs — instead of a separate f32 read +
    cast launch.  The earlier block takes the copy only if its dout IS that dx (same storage, shape,
    strides, version: the handoff holds dx, so its memory cannot have been reused)."""
    __slots__ = ("scale", "dx", "dx16", "ver")

    def __init__(self, scale):
        self.scale, self.dx, self.dx16, self.ver = scale, None, None, -1

    def put(self, dx, dx16):
        self.dx, self.dx16, self.ver = dx, dx16, dx._version

    def take(self, dout):
        dx, dx16 = self.dx, self.dx16
        self.dx = self.dx16 = None
        if (dx is None or dout.data_ptr() != dx.data_ptr() or dout.shape != dx.shape or dout.stride() != dx.stride()
                or dout._version != self.ver):
            return None
        return dx16


# (module switches the tests turn off to compare against the per-block launches)
_DEFER_REDUCTIONS = True
# with the reductions deferred, the blocks' weight gradients too: one grouped launch for the stage
_DEFER_WGRAD = True
# a deferred weight gradient known to start from zero is stored, not added (FlatParams.claim_fresh)
_STORE_FRESH = True


def _stage_deferral(blocks, flat):
    """A DeferredGrads the stage's blocks share, or None: the LayerNorm gamma / beta and bias-table
    gradient reductions and the weight gradients of every block then run as batched launches when the
    backward reaches the stage's first block (always the last of them, and present in the graph whenever
    its parameters train).  With a gradient reducer the stage's blocks report their parameters final
    together, at that flush (a bucket's exchange starts then, instead of block by block)."""
    if not _DEFER_REDUCTIONS or not torch.is_grad_enabled():
        return None
    if not any(p.requires_grad for p in blocks[0].parameters()):
        return None
    d = K.DeferredGrads(len(blocks))
    d.blocks = list(blocks)
    return d


def _run_blocks(blocks, x, geo, flat, scales, tiles=None):
    """The blocks of one stage in order; scales [(dp1, dp2)] per block (None entries in eval);
    tiles: per block the (forward, backward) bias tiles built ahead (_prebuild_bias_tiles) or None."""
    links = [None] + [_Handoff(scales[j - 1][1]) if _HANDOFF else None for j in range(1, len(blocks))]
    red = _stage_deferral(blocks, flat)
    for j, blk in enumerate(blocks):
        dp1, dp2 = scales[j]
        x = _SwinBlockFn.apply(x, blk, geo, flat, dp1, dp2, links[j], links[j + 1] if j + 1 < len(blocks) else None,
                               tiles[j] if tiles is not None else None, (red, j == 0) if red is not None else None,
                               *blk.parameters())
    return x


def _bias_tiles(blk, geo):
    """The block's relative-position bias expanded to per-(mask pattern, head) score tiles
    (video_swin_ori.py:171-174 gather + the shifted-window mask), forward and backward forms: fp16
    for the fused head-pair kernels, f32 for odd head counts."""
    nH = blk.num_heads
    shifted = geo.shifted and any(s > 0 for s in blk.shift_size)
    region, n_pat = (geo.region, geo.n_pat) if shifted else (None, 1)
    dt = torch.float16 if nH % 2 == 0 else torch.float32
    dev = blk.attn.relative_position_bias_table.device
    bias_f = torch.empty(K.wattn_bias_elems(n_pat, nH), device=dev, dtype=dt)
    bias_b = torch.empty(K.wattn_bias_elems(n_pat, nH), device=dev, dtype=dt)
    K.wattn_bias_build(blk.attn.relative_position_bias_table, blk.attn.relative_position_index, geo.n, nH, region,
                       n_pat, bias_f, bias_b)
    return bias_f, bias_b


def _prebuild_bias_tiles(stages, dev):
    """Every block's bias tiles for the whole forward, built in stage order on an aux stream (they
    depend only on the parameters, which the stream sees after waiting on the current one): the 24
    small build launches leave the forward's critical path and overlap the patch embedding / earlier
    stages.  stages: [(blocks, geo)]; returns per stage (tiles per block, event the stage waits on)."""
    main = torch.cuda.current_stream(dev)
    s = aux_stream(dev, "swin_bias")
    s.wait_stream(main)
    out = []
    with torch.cuda.stream(s):
        for blocks, geo in stages:
            tiles = [_bias_tiles(blk, geo) for blk in blocks]
            ev = torch.cuda.Event()
            ev.record(s)
            out.append((tiles, ev))
    return out


class _SwinBlockFn(torch.autograd.Function):
    """One SwinTransformerBlock3D (video_swin_ori.py:248-306) forward / backward."""

    @staticmethod
    def forward(ctx, x, blk, geo, flat, dp1, dp2, up, down, tiles, red, *params):
        """up: the _Handoff this block's backward fills for the block before it; down: the one the
        block after it fills for this block (either None); tiles: prebuilt (forward, backward) bias
        tiles or None (built here); red: (the stage's DeferredGrads, is the stage's first block) or
        None (reductions launched in place)."""
        C, nH, n, M = blk.dim, blk.num_heads, geo.n, geo.M
        at = blk.attn
        shifted = geo.shifted and any(s > 0 for s in blk.shift_size)
        wmap = geo.win2sp_shift if shifted else geo.win2sp
        win_pat = geo.win_pat if shifted else None
        dev = x.device
        fused = nH % 2 == 0
        bias_f, bias_b = tiles if tiles is not None else _bias_tiles(blk, geo)
        Mw = geo.M_win   # window-order rows (incl. the padded positions of a partial window)
        xw, m1, r1 = K.layernorm(x, blk.norm1.weight, blk.norm1.bias, 1e-5, in_map=wmap, rows=Mw)
        c = (C // nH) ** -0.5 * LOG2E
        o = torch.empty(Mw, C, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(geo.n_win, nH, 160, device=dev)
        if fused:
            # QKV projection fused with the attention (csrc/window_fused.hip); qkv is still written
            # for the backward
            qkv = torch.empty(Mw, 3 * C, dtype=torch.bfloat16, device=dev)
            K.wattn_qkv_fwd(xw, flat.w16(at.qkv.weight), at.qkv.bias, c, bias_f, win_pat, qkv, o, lse, geo.n_win, n,
                            nH, win_order=geo.win_order if shifted else None)
        else:   # odd head counts (the fused kernel takes heads in pairs; not Swin-B)
            qkv = K.linear(xw, flat.w16(at.qkv.weight), at.qkv.bias, scale_cols=C, scale_val=c)
            K.wattn_fwd_grouped(qkv, bias_f, geo.groups_shift if shifted else geo.groups, o, lse, geo.n_win, n, nH)
        x_mid = torch.empty(M, C, device=dev)
        K.linear(o, flat.w16(at.proj.weight), at.proj.bias, out=x_mid, resid=x, c_map=wmap, row_scale=dp1,
                 rows_per_scale=geo.win_rows_per_clip)
        h2, m2, r2 = K.layernorm(x_mid, blk.norm2.weight, blk.norm2.bias, 1e-5)
        pre = torch.empty(M, 4 * C, dtype=torch.bfloat16, device=dev)
        g = K.linear(h2, flat.w16(blk.mlp.fc1.weight), blk.mlp.fc1.bias, gelu=True, pre_out=pre)
        out = torch.empty(M, C, device=dev)
        K.linear(g, flat.w16(blk.mlp.fc2.weight), blk.mlp.fc2.bias, out=out, resid=x_mid, row_scale=dp2,
                 rows_per_scale=geo.rows_per_clip)
        if any(t.requires_grad for t in (x,) + params):
            ctx.save = (x, xw, m1, r1, qkv, o, lse, x_mid, h2, m2, r2, pre, g, bias_b)
            ctx.blk, ctx.geo, ctx.flat, ctx.dp1, ctx.dp2 = blk, geo, flat, dp1, dp2
            ctx.wmap, ctx.win_pat, ctx.up, ctx.down, ctx.red = wmap, win_pat, up, down, red
            ctx.sp2win = geo.sp2win_shift if shifted else geo.sp2win
        return out

    @staticmethod
    def backward(ctx, dout):
        x, xw, m1, r1, qkv, o, lse, x_mid, h2, m2, r2, pre, g, bias_b = ctx.save
        blk, geo, flat, dp1, dp2, wmap = ctx.blk, ctx.geo, ctx.flat, ctx.dp1, ctx.dp2, ctx.wmap
        at = blk.attn
        C, nH, n, M = blk.dim, blk.num_heads, geo.n, geo.M
        rpc = geo.rows_per_clip
        red, flush = ctx.red if ctx.red is not None else (None, False)
        dout16 = ctx.down.take(dout) if ctx.down is not None else None
        dout = dout.contiguous()
        # MLP branch: y = x_mid + s2 * fc2(gelu(fc1(LN2(x_mid)))).  The branch's GEMMs read the
        # DropPath-scaled gradient as one bf16 copy (the A operand of both dW and dX), written by the
        # next block's LN1 backward when there is one
        if dout16 is None:
            dout16 = K.scale_cast_bf16(dout, dp2, rpc)
        _wgrad(flat, blk.mlp.fc2, dout16, g, red)
        dpre = K.linear_dx(dout16, flat.w16(blk.mlp.fc2.weight), out_f32=False, dgelu_pre=pre)
        del g, pre, dout16
        _wgrad(flat, blk.mlp.fc1, dpre, h2, red)
        # the LayerNorms' input gradients arrive as bf16 GEMM outputs (as under the reference's
        # autocast, where a bf16 linear's grad_input is bf16): half the bytes of the LN backward's dy;
        # rows of >= 1024 columns keep f32 (the LN backward's bf16 loads measured slower there)
        dh2 = K.linear_dx(dpre, flat.w16(blk.mlp.fc1.weight), out_f32=C >= _LN_F32_WIDE)
        del dpre, h2
        dx_mid = torch.empty_like(x_mid)
        # attention branch input gradient s1 * dx_mid, as bf16 in window order (rows of o / qkv)
        # (window order; padded positions carry no gradient: the reference crops them, :292-293)
        dmid16 = (torch.zeros if geo.padded else torch.empty)(geo.M_win, C, dtype=torch.bfloat16, device=dout.device)
        K.layernorm_bwd(dh2, x_mid, m2, r2, blk.norm2.weight, dx_mid, dres=dout,
                        dw=_g(flat, blk.norm2.weight), db=_g(flat, blk.norm2.bias),
                        dx16=dmid16, dx16_map=ctx.sp2win, dx_scale=dp1, dx_scale_rps=rpc, defer=red)
        del dh2
        # attention branch: x_mid = x + s1 * unwindow(proj(attn(qkv(LN1(window(x))))))
        _wgrad(flat, at.proj, dmid16, o, red)
        do = K.linear_dx(dmid16, flat.w16(at.proj.weight), out_f32=False)
        del dmid16
        dqkv = torch.empty_like(qkv)
        dbp = torch.empty(K.wattn_dbias_part_elems(geo.n_win, nH, geo.ws), device=dout.device)
        K.wattn_bwd(qkv, o, do, lse, bias_b, ctx.win_pat, dqkv, dbp, geo.n_win, n, nH, geo.ws)
        del do, o
        gt = _g(flat, at.relative_position_bias_table)
        if gt is not None:
            K.wattn_dbias(dbp, geo.n_win, nH, geo.ws, _bin_rows(at, geo.ws), gt, defer=red)
        del dbp
        _wgrad(flat, at.qkv, dqkv, xw, red)
        dxw = K.linear_dx(dqkv, flat.w16(at.qkv.weight), out_f32=C >= _LN_F32_WIDE)
        del dqkv, qkv, xw
        dx = torch.empty_like(x)
        up = ctx.up
        # for the previous block: dx as bf16 times its dp2, in token order (rows r of this LN are in
        # window order, clip-major: the scale index is r / rows-per-clip in window order)
        dx16 = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if up is not None else None
        K.layernorm_bwd(dxw, x, m1, r1, blk.norm1.weight, dx, in_map=wmap, dres=dx_mid,
                        dw=_g(flat, blk.norm1.weight), db=_g(flat, blk.norm1.bias), dx16=dx16,
                        dx16_map=wmap if up is not None else None, dx_scale=up.scale if up is not None else None,
                        dx_scale_rps=geo.win_rows_per_clip, defer=red)
        if up is not None:
            up.put(dx, dx16)
        if flush:
            red.flush(dx)   # the stage's deferred LayerNorm / bias-table gradient sums
        ctx.save = ctx.up = ctx.down = ctx.red = None
        if red is None:
            flat.notify(blk.parameters())
        elif flush:   # every block of the stage is final only now (their gradients were deferred)
            for b in red.blocks:
                flat.notify(b.parameters())
        group = getattr(blk, "_lrce_group", None)
        if group is not None and flat.early_update is not None:
            # this stage's gradients are final: its optimizer update runs on the decoder's weight-
            # gradient stream (joined at the end of backward by the decoder's stream anchor) while
            # the earlier stages' backward continues here; it touches only this stage's weights
            main = torch.cuda.current_stream(dout.device)
            s = aux_stream(dout.device, "decoder_wgrad")
            s.wait_stream(main)
            with torch.cuda.stream(s):
                flat.group_done(group)
        return (dx, None, None, None, None, None, None, None, None, None) + (None,) * len(ctx.needs_input_grad[10:])


class _PatchMergeFn(torch.autograd.Function):
    """PatchMerging (video_swin_ori.py:321-342): 2x2 gather + LN(4C) fused, then the 4C->2C GEMM."""

    @staticmethod
    def forward(ctx, x, pm, geo, flat, *params):
        C = pm.dim
        Mo = geo.M_merged
        xl, mean, rstd = K.layernorm(x, pm.norm.weight, pm.norm.bias, 1e-5, in_map=geo.merge_map, nseg=4, rows=Mo,
                                     cols=4 * C)
        y = K.linear(xl, flat.w16(pm.reduction.weight), out_f32=True)
        ctx.save = (x, xl, mean, rstd)
        ctx.pm, ctx.geo, ctx.flat = pm, geo, flat
        return y

    @staticmethod
    def backward(ctx, dy):
        x, xl, mean, rstd = ctx.save
        pm, geo, flat = ctx.pm, ctx.geo, ctx.flat
        dy16 = K.scale_cast_bf16(dy.contiguous().view(-1, dy.shape[-1]))
        gw = _g(flat, pm.reduction.weight)
        if gw is not None:
            K.linear_dw(dy16, xl, gw)
        dxl = K.linear_dx(dy16, flat.w16(pm.reduction.weight), out_f32=4 * pm.dim >= _LN_F32_WIDE)
        dx = torch.empty_like(x)
        K.layernorm_bwd(dxl, x, mean, rstd, pm.norm.weight, dx, in_map=geo.merge_map, nseg=4, rows=geo.M_merged,
                        cols=4 * pm.dim, dw=_g(flat, pm.norm.weight), db=_g(flat, pm.norm.bias))
        ctx.save = None
        flat.notify(pm.parameters())
        return (dx, None, None, None) + (None,) * len(ctx.needs_input_grad[4:])


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ln, flat, eps, *params):
        y, mean, rstd = K.layernorm(x, ln.weight, ln.bias, eps, out_f32=True)
        ctx.save = (x, mean, rstd)
        ctx.ln, ctx.flat = ln, flat
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd = ctx.save
        dx = torch.empty_like(x)
        K.layernorm_bwd(dy.contiguous(), x, mean, rstd, ctx.ln.weight, dx, dw=_g(ctx.flat, ctx.ln.weight),
                        db=_g(ctx.flat, ctx.ln.bias))
        ctx.flat.notify(ctx.ln.parameters())
        return (dx, None, None, None) + (None,) * len(ctx.needs_input_grad[4:])


# ----------------------------------------------------------------------------------- backbone
class SwinTransformer3D(nn.Module):
    """Swin3D backbone; parameter tree of video_swin_ori.py:485-571 (frozen_stages=-1, patch_norm)."""

    def __init__(self, patch_size=(2, 4, 4), in_chans=3, embed_dim=128, depths=(2, 2, 18, 2), num_heads=(4, 8, 16, 32),
                 window_size=(8, 7, 7), drop_path_rate=0.2, patch_norm=True, **unused):
        super().__init__()
        if not patch_norm:
            raise ValueError("patch_norm=False is not used by the LRCE extractor")
        self.embed_dim, self.window_size, self.patch_size = embed_dim, tuple(window_size), tuple(patch_size)
        self.depths, self.num_heads = tuple(depths), tuple(num_heads)
        self.patch_embed = PatchEmbed3D(patch_size, in_chans, embed_dim)
        self.pos_drop = nn.Dropout(0.0)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]
        self.layers = nn.ModuleList()
        for i, (dep, nh) in enumerate(zip(depths, num_heads)):
            self.layers.append(BasicLayer(embed_dim * 2 ** i, dep, nh, self.window_size,
                                          dpr[sum(depths[:i]):sum(depths[:i + 1])], i < len(depths) - 1))
        self.num_features = embed_dim * 2 ** (len(depths) - 1)
        self.norm = nn.LayerNorm(self.num_features)
        # split backward (data parallel, E2EBase.split_swin_stage): the input of stage split_at enters it
        # as a detached leaf, so one backward call ends there and backward_below_split() continues
        self.split_at = None
        self._split_mid = None
        # stage i > 0 is final once its first block's backward is done (the backward runs the last
        # stage first): that block reports the stage's optimizer group (E2EBase.optimizer_groups)
        for i, layer in enumerate(self.layers):
            object.__setattr__(layer.blocks[0], "_lrce_group", f"swin{i}" if i > 0 else None)

    def forward_tokens(self, clips, layout="BSTCHW", normalize=True):
        """clips (B,S,T,3,H,W) f32 in [0,1] (normalised in-kernel) or (B,3,T,H,W) already normalised.
        Returns (features f32 [n_clips*D'*H'*W', C_out], (n_clips, D', H', W'))."""
        flat = ensure(self)
        dev = clips.device
        x = _PatchEmbedFn.apply(clips, self.patch_embed, flat, layout, normalize, *self.patch_embed.parameters())
        if layout == "BSTCHW":
            B, S, T, _, H, W = clips.shape
            nc = B * S
        else:
            B, _, T, H, W = clips.shape
            nc = B
        D, H, W = (T + 1) // 2, H // 4, W // 4
        scales = _drop_path_scales(self, nc, dev)
        geos, (h, w) = [], (H, W)
        for layer in self.layers:
            geos.append(stage_geometry(nc, D, h, w, self.window_size, dev))
            if layer.downsample is not None:
                h, w = (h + 1) // 2, (w + 1) // 2
        pre = (_prebuild_bias_tiles([(list(layer.blocks), g) for layer, g in zip(self.layers, geos)], dev)
               if dev.type == "cuda" else None)
        bi = 0
        for li, layer in enumerate(self.layers):
            if li == self.split_at and torch.is_grad_enabled() and x.requires_grad:
                x_leaf = x.detach().requires_grad_(True)
                self._split_mid = (x, x_leaf)
                x = x_leaf
            geo = geos[li]
            nb = len(layer.blocks)
            tiles = None
            if pre is not None:
                tiles, ev = pre[li]
                torch.cuda.current_stream(dev).wait_event(ev)
            blocks = list(layer.blocks)
            x = _run_blocks(blocks, x, geo, flat,
                            scales[bi:bi + len(blocks)] if scales is not None else [(None, None)] * len(blocks),
                            tiles[:len(blocks)] if tiles is not None else None)
            bi += nb
            if layer.downsample is not None:
                x = _PatchMergeFn.apply(x, layer.downsample, geo, flat, *layer.downsample.parameters())
                H, W = (H + 1) // 2, (W + 1) // 2
        x = _LayerNormFn.apply(x, self.norm, flat, 1e-5, *self.norm.parameters())
        return x, (nc, D, H, W)

    def backward_below_split(self):
        """Second part of a split Swin backward: stages below split_at (and the patch embedding) from
        the gradient the first part left on the stage input.  No-op when the forward made no split
        (frozen lower stages / patch embedding, or a forward without gradients)."""
        if self._split_mid is None:
            return
        x, x_leaf = self._split_mid
        self._split_mid = None
        if x_leaf.grad is None:
            return
        torch.autograd.backward([x], [x_leaf.grad])

    def forward_stage(self, i, x_cl, depth=None):
        """Run stage i (its first `depth` blocks, all by default, then PatchMerging) on channels-last
        x_cl (nc, D, H, W, C) f32; returns the next stage's channels-last input.  (Test /
        introspection entry: per-stage parity fixtures.)"""
        flat = ensure(self)
        nc, D, H, W, C = x_cl.shape
        geo = stage_geometry(nc, D, H, W, self.window_size, x_cl.device)
        x = x_cl.reshape(-1, C).contiguous()
        layer = self.layers[i]
        blocks = list(layer.blocks)[:depth]
        scales = [(_drop_path_scale(blk.drop_path, nc, x.device, self.training),
                   _drop_path_scale(blk.drop_path, nc, x.device, self.training)) for blk in blocks]
        x = _run_blocks(blocks, x, geo, flat, scales)
        if layer.downsample is not None:
            x = _PatchMergeFn.apply(x, layer.downsample, geo, flat, *layer.downsample.parameters())
            H, W = (H + 1) // 2, (W + 1) // 2
        return x.view(nc, D, H, W, -1)

    def forward(self, x):
        """Reference signature (video_swin_ori.py:674-687): x (B,3,T,H,W) normalised -> (B,C,D',H',W')."""
        feats, (nc, D, H, W) = self.forward_tokens(x.contiguous(), layout="BCTHW", normalize=False)
        return feats.view(nc, D, H, W, -1).permute(0, 4, 1, 2, 3)

    def train(self, mode=True):
        # the reference's override returns None (video_swin_ori.py:689-692); keep nn.Module semantics
        return super().train(mode)
