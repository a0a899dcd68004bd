"""CPU ORACLE (test infrastructure only) — a functional fp32 restatement of the reference LRCE
forward pass: Video Swin-B 3D extractor -> BERT-base text encoder -> recurrent cross-modal
decoder -> answer head.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / CPU baseline.  The product path (vqa-lrce-kbs-2023_amd/lrce) never calls it.

Parity pinning: tests/golden/make_golden.py imports the reference itself (/root/reference, with
stand-ins for absent packages) in the survey container, runs it on the deterministic weight
recipe (oracle/weights.py) and commits its outputs under tests/golden/; tests/test_oracle.py
checks this restatement against them.  Third-party arithmetic on the path (HF BertModel,
torch nn.TransformerDecoder) is restated from their published algorithms and pinned only by those
same fixtures (the reference has no tests of its own — SURVEY.md §4).

Every function cites the reference file:line it restates (paths relative to the reference root).
Tensors are channels-last inside Swin: (B, D, H, W, C).
"""
import math
from functools import lru_cache

import torch
import torch.nn.functional as F

IMAGENET_MEAN = (0.485, 0.456, 0.406)   # lrce/feature_extractor/video.py:35
IMAGENET_STD = (0.229, 0.224, 0.225)

SWIN_CFG = dict(embed_dim=128, depths=(2, 2, 18, 2), heads=(4, 8, 16, 32), patch=(2, 4, 4),
                window=(8, 7, 7))      # lrce/feature_extractor/video.py:10-18
LN_EPS_SWIN = 1e-5                     # nn.LayerNorm default (video_swin_ori.py:234,244,319,569)
LN_EPS_BERT = 1e-12                    # BertConfig.layer_norm_eps
LN_EPS_FUSION = 1e-12                  # fusionv3.py:14,18; embedding.py:15,42


def _ln(x, sd, p, eps):
    return F.layer_norm(x, (x.shape[-1],), sd[p + "weight"], sd[p + "bias"], eps)


def _lin(x, sd, p, bias=True):
    return F.linear(x, sd[p + "weight"], sd[p + "bias"] if bias else None)


# ----------------------------------------------------------------------------- Swin 3D
def normalize_clip(clip):
    """video.py:35 — torchvision Normalize over the channel dim (-3) of (B,T,3,H,W)."""
    m = torch.tensor(IMAGENET_MEAN, dtype=clip.dtype).view(3, 1, 1)
    s = torch.tensor(IMAGENET_STD, dtype=clip.dtype).view(3, 1, 1)
    return (clip - m) / s


def patch_embed(x, sd, p):
    """video_swin_ori.py:464-482.  x (B,3,T,H,W) already normalized.  Zero-pad W,H,T to multiples
    of the patch (after normalization), conv3d k=s=(2,4,4) + bias, LayerNorm(128).
    Returns channels-last (B,D,H,W,C)."""
    pt, ph, pw = SWIN_CFG["patch"]
    _, _, T, H, W = x.shape
    x = F.pad(x, (0, (-W) % pw, 0, (-H) % ph, 0, (-T) % pt))
    y = F.conv3d(x, sd[p + "proj.weight"], sd[p + "proj.bias"], stride=(pt, ph, pw))
    y = y.permute(0, 2, 3, 4, 1)
    return _ln(y, sd, p + "norm.", LN_EPS_SWIN)


def clamp_window(x_size, window, shift):
    """video_swin_ori.py:91-104 (get_window_size): a dim no larger than the window uses the whole
    dim and gets zero shift."""
    ws, ss = list(window), list(shift)
    for i in range(3):
        if x_size[i] <= window[i]:
            ws[i] = x_size[i]
            ss[i] = 0
    return tuple(ws), tuple(ss)


def relative_position_index(window):
    """video_swin_ori.py:133-148 — pairwise relative index into the (2Wd-1)(2Wh-1)(2Ww-1) table
    for the UNCLAMPED window; forward slices [:N,:N] (:171)."""
    wd, wh, ww = window
    g = torch.stack(torch.meshgrid(torch.arange(wd), torch.arange(wh), torch.arange(ww), indexing="ij")).flatten(1)
    rel = (g[:, :, None] - g[:, None, :]).permute(1, 2, 0)
    rel = rel + torch.tensor([wd - 1, wh - 1, ww - 1])
    return rel[..., 0] * (2 * wh - 1) * (2 * ww - 1) + rel[..., 1] * (2 * ww - 1) + rel[..., 2]


def partition(x, ws):
    """video_swin_ori.py:60-72.  (B,D,H,W,C) -> (B*nW, wd*wh*ww, C), windows ordered (d,h,w)."""
    B, D, H, W, C = x.shape
    x = x.view(B, D // ws[0], ws[0], H // ws[1], ws[1], W // ws[2], ws[2], C)
    return x.permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(-1, ws[0] * ws[1] * ws[2], C)


def unpartition(win, ws, B, D, H, W):
    """video_swin_ori.py:75-88."""
    x = win.view(B, D // ws[0], H // ws[1], W // ws[2], ws[0], ws[1], ws[2], -1)
    return x.permute(0, 1, 4, 2, 5, 3, 6, 7).reshape(B, D, H, W, -1)


@lru_cache(maxsize=None)
def shift_mask(D, H, W, ws, ss):
    """video_swin_ori.py:346-359 (compute_mask).  Region labels over the padded volume, assigned
    by the reference's 3x3x3 slice loop (an empty slice still advances the label), then -100.0
    between tokens of different regions inside each window."""
    img = torch.zeros((1, D, H, W, 1))
    cnt = 0
    for d in (slice(-ws[0]), slice(-ws[0], -ss[0]), slice(-ss[0], None)):
        for h in (slice(-ws[1]), slice(-ws[1], -ss[1]), slice(-ss[1], None)):
            for w in (slice(-ws[2]), slice(-ws[2], -ss[2]), slice(-ss[2], None)):
                img[:, d, h, w, :] = cnt
                cnt += 1
    mw = partition(img, ws).squeeze(-1)
    diff = mw.unsqueeze(1) - mw.unsqueeze(2)
    return torch.where(diff != 0, torch.tensor(-100.0), torch.tensor(0.0))


def window_attention(xw, sd, p, nH, mask):
    """video_swin_ori.py:158-189.  xw (B_,N,C)."""
    B_, N, C = xw.shape
    hd = C // nH
    qkv = _lin(xw, sd, p + "qkv.").reshape(B_, N, 3, nH, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0] * hd ** -0.5, qkv[1], qkv[2]
    att = q @ k.transpose(-2, -1)
    idx = relative_position_index(SWIN_CFG["window"])[:N, :N].reshape(-1)
    bias = sd[p + "relative_position_bias_table"][idx].reshape(N, N, nH).permute(2, 0, 1)
    att = att + bias.unsqueeze(0)
    if mask is not None:
        nW = mask.shape[0]
        att = att.view(B_ // nW, nW, nH, N, N) + mask.view(1, nW, 1, N, N)
        att = att.view(B_, nH, N, N)
    att = att.softmax(-1)
    out = (att @ v).transpose(1, 2).reshape(B_, N, C)
    return _lin(out, sd, p + "proj.")


def swin_block(x, sd, p, nH, shift_req, mask):
    """video_swin_ori.py:248-306 (forward_part1/part2/forward), eval mode (DropPath = identity)."""
    B, D, H, W, C = x.shape
    ws, ss = clamp_window((D, H, W), SWIN_CFG["window"], shift_req)
    h = _ln(x, sd, p + "norm1.", LN_EPS_SWIN)
    pd, pb, pr = (-D) % ws[0], (-H) % ws[1], (-W) % ws[2]
    h = F.pad(h, (0, 0, 0, pr, 0, pb, 0, pd))
    _, Dp, Hp, Wp, _ = h.shape
    shifted = any(s > 0 for s in ss)
    if shifted:
        h = torch.roll(h, shifts=(-ss[0], -ss[1], -ss[2]), dims=(1, 2, 3))
    a = window_attention(partition(h, ws), sd, p + "attn.", nH, mask if shifted else None)
    h = unpartition(a, ws, B, Dp, Hp, Wp)
    if shifted:
        h = torch.roll(h, shifts=ss, dims=(1, 2, 3))
    h = h[:, :D, :H, :W, :]
    x = x + h
    m = _ln(x, sd, p + "norm2.", LN_EPS_SWIN)
    m = _lin(F.gelu(_lin(m, sd, p + "mlp.fc1.")), sd, p + "mlp.fc2.")
    return x + m


def patch_merging(x, sd, p):
    """video_swin_ori.py:321-342: 2x2 gather in order (0,0),(1,0),(0,1),(1,1) -> LN(4C) -> Linear(4C,2C)."""
    _, _, H, W, _ = x.shape
    if H % 2 or W % 2:
        x = F.pad(x, (0, 0, 0, W % 2, 0, H % 2))
    x = torch.cat([x[:, :, 0::2, 0::2], x[:, :, 1::2, 0::2], x[:, :, 0::2, 1::2], x[:, :, 1::2, 1::2]], -1)
    return _lin(_ln(x, sd, p + "norm.", LN_EPS_SWIN), sd, p + "reduction.", bias=False)


def swin_stage(x, sd, p, depth, nH, has_merge):
    """video_swin_ori.py:420-440 (BasicLayer.forward): mask from the stage-level clamped window
    and shift (shift = window//2 on odd blocks), then blocks, then PatchMerging."""
    B, D, H, W, C = x.shape
    win = SWIN_CFG["window"]
    half = tuple(i // 2 for i in win)
    ws, ss = clamp_window((D, H, W), win, half)
    Dp, Hp, Wp = (math.ceil(D / ws[0]) * ws[0], math.ceil(H / ws[1]) * ws[1], math.ceil(W / ws[2]) * ws[2])
    mask = shift_mask(Dp, Hp, Wp, ws, ss)
    for i in range(depth):
        x = swin_block(x, sd, f"{p}blocks.{i}.", nH, (0, 0, 0) if i % 2 == 0 else half, mask)
    if has_merge:
        x = patch_merging(x, sd, p + "downsample.")
    return x


def swin_forward(x, sd, p="video_extractor.swin."):
    """video_swin_ori.py:674-687.  x (B,3,T,H,W) normalized -> (B,D,H,W,1024) channels-last."""
    x = patch_embed(x, sd, p + "patch_embed.")
    for i, (dep, nH) in enumerate(zip(SWIN_CFG["depths"], SWIN_CFG["heads"])):
        x = swin_stage(x, sd, f"{p}layers.{i}.", dep, nH, i < 3)
    return _ln(x, sd, p + "norm.", LN_EPS_SWIN)


def video_extractor(clips, sd):
    """video.py:28-43.  clips (B,S,T,3,H,W) -> (B,S,(T+1)//2,(H//32)*(W//32),1024)."""
    B, S, T, _, H, W = clips.shape
    outs = []
    for i in range(S):
        c = normalize_clip(clips[:, i])
        f = swin_forward(c.transpose(1, 2), sd)
        outs.append(f.reshape(B, f.shape[1], f.shape[2] * f.shape[3], f.shape[4]))
    return torch.stack(outs, 1)


# ----------------------------------------------------------------------------- BERT-base
def bert(ids, mask, types, sd, p="text_extractor.bert.", n_layers=12, n_heads=12):
    """text.py:11-17 -> HF BertModel(bert-base-uncased).last_hidden_state (transformers 4.20.1
    published algorithm): embeddings(word+position+token_type) -> LN(1e-12) -> 12 post-norm
    layers [MHA with additive key-padding mask, GELU(erf) FFN].  The pooler is computed by the
    reference but unused (text.py:12-17), so it is not restated."""
    B, L = ids.shape
    e = p + "embeddings."
    # word embeddings are nn.Embedding(vocab, 768, padding_idx=pad_token_id=0): row 0 gets no gradient
    x = F.embedding(ids, sd[e + "word_embeddings.weight"], padding_idx=0) \
        + sd[e + "position_embeddings.weight"][:L].unsqueeze(0) + sd[e + "token_type_embeddings.weight"][types]
    x = _ln(x, sd, e + "LayerNorm.", LN_EPS_BERT)
    add = (1.0 - mask.to(x.dtype))[:, None, None, :] * torch.finfo(x.dtype).min
    hd = x.shape[-1] // n_heads
    for i in range(n_layers):
        q_ = f"{p}encoder.layer.{i}."
        def heads(t):
            return t.view(B, L, n_heads, hd).transpose(1, 2)
        q = heads(_lin(x, sd, q_ + "attention.self.query."))
        k = heads(_lin(x, sd, q_ + "attention.self.key."))
        v = heads(_lin(x, sd, q_ + "attention.self.value."))
        s = (q @ k.transpose(-1, -2)) / math.sqrt(hd) + add
        ctx = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, L, -1)
        h = _ln(_lin(ctx, sd, q_ + "attention.output.dense.") + x, sd, q_ + "attention.output.LayerNorm.", LN_EPS_BERT)
        f = _lin(F.gelu(_lin(h, sd, q_ + "intermediate.dense.")), sd, q_ + "output.dense.")
        x = _ln(f + h, sd, q_ + "output.LayerNorm.", LN_EPS_BERT)
    return x


# ----------------------------------------------------------------------------- LRCE fusion
def video_pos_embed(v, sd, p):
    """embedding.py:47-63.  v (B,S,Tg,49,768) -> (B,S,Tg*50,768)."""
    B, S, Tg, F_, C = v.shape
    cls = sd[p + "emb_cls"].expand(B, S, Tg, 1, C)
    x = torch.cat([cls, v], 3)
    x = x + sd[p + "emb_pos"] + sd[p + "emb_len"] + sd[p + "emb_clip"]
    x = _ln(x, sd, p + "layer_norm.", LN_EPS_FUSION)
    return x.reshape(B, S, Tg * (1 + F_), C)


def text_pos_embed(t, sd, p):
    """embedding.py:17-23.  t (B,L,768) -> (B,L+1,768)."""
    B = t.shape[0]
    x = torch.cat([sd[p + "emb_cls"].expand(B, 1, -1), t], 1) + sd[p + "emb_pos"]
    return _ln(x, sd, p + "layer_norm.", LN_EPS_FUSION)


def decoder_layer(x, mem, sd, p, n_heads=12):
    """torch nn.TransformerDecoderLayer (post-norm, batch_first, GELU, eps 1e-12) as configured at
    fusionv3.py:8-17, eval mode.  Self-attention over a single query token reduces exactly to
    out_proj(v_proj(x)) (softmax over one key == 1)."""
    E = x.shape[-1]
    Wi, bi = sd[p + "self_attn.in_proj_weight"], sd[p + "self_attn.in_proj_bias"]
    if x.shape[1] == 1:
        sa = F.linear(x, Wi[2 * E:], bi[2 * E:])
    else:  # general form (not reached by the reference, kept for completeness)
        sa = _mha(x, x, Wi, bi, n_heads)
    sa = _lin(sa, sd, p + "self_attn.out_proj.")
    x = _ln(x + sa, sd, p + "norm1.", LN_EPS_FUSION)
    ca = _mha(x, mem, sd[p + "multihead_attn.in_proj_weight"], sd[p + "multihead_attn.in_proj_bias"], n_heads)
    ca = _lin(ca, sd, p + "multihead_attn.out_proj.")
    x = _ln(x + ca, sd, p + "norm2.", LN_EPS_FUSION)
    f = _lin(F.gelu(_lin(x, sd, p + "linear1.")), sd, p + "linear2.")
    return _ln(x + f, sd, p + "norm3.", LN_EPS_FUSION)


def _mha(q_in, kv_in, W, b, n_heads):
    E = q_in.shape[-1]
    hd = E // n_heads
    B, Lq, _ = q_in.shape
    Lk = kv_in.shape[1]
    q = F.linear(q_in, W[:E], b[:E]).view(B, Lq, n_heads, hd).transpose(1, 2)
    k = F.linear(kv_in, W[E:2 * E], b[E:2 * E]).view(B, Lk, n_heads, hd).transpose(1, 2)
    v = F.linear(kv_in, W[2 * E:], b[2 * E:]).view(B, Lk, n_heads, hd).transpose(1, 2)
    s = (q / math.sqrt(hd)) @ k.transpose(-1, -2)
    return (s.softmax(-1) @ v).transpose(1, 2).reshape(B, Lq, E)


def fusion_transformer(video, text, sd, p="fusion_model.fusion_transformer.", n_layers=12):
    """fusionv3.py:27-51.  video (B,S,150,768), text (B,L+1,768) -> (B,1,768).
    texts_attention_mask is accepted by the reference but never used (no key-padding mask)."""
    B, S = video.shape[:2]
    s = sd[p + "summarization_token"].expand(B, 1, -1)
    for i in range(S):
        mem = torch.cat([video[:, i], text], 1)
        o = s
        for k in range(n_layers):
            o = decoder_layer(o, mem, sd, f"{p}transformer.layers.{k}.")
        s = _ln(s + o, sd, p + "fusion_layer_norm.", LN_EPS_FUSION)
    return s


def fusion_video(video, sd, p="fusion_model.fusion_transformer.", n_layers=12):
    """fusionv3.py:70-88 (FusionVideo): the recurrent decoder with the step's video tokens as the only
    memory.  video (B,S,150,768) -> (B,1,768)."""
    B, S = video.shape[:2]
    s = sd[p + "summarization_token"].expand(B, 1, -1)
    for i in range(S):
        o = s
        for k in range(n_layers):
            o = decoder_layer(o, video[:, i], sd, f"{p}transformer.layers.{k}.")
        s = _ln(s + o, sd, p + "fusion_layer_norm.", LN_EPS_FUSION)
    return s


def lrce_mc_sim(video_feats, text_feats, sd, p="fusion_model."):
    """fusionv3.py:301-333 (LRCEMultipleChoiceSim.forward), eval mode: cosine between the projected
    mean text embedding of each choice and the FusionVideo summary.  text (B,5,L,768) -> (B,5)."""
    B, n_mc = text_feats.shape[:2]
    v = _lin(video_feats, sd, p + "projection_layer.")
    v = video_pos_embed(v, sd, p + "video_pos_embed.")
    t = text_pos_embed(text_feats.flatten(0, 1), sd, p + "question_pos_embed.")
    tf = _lin(t.mean(1), sd, p + "text_projection.")
    vf = fusion_video(v, sd).expand(-1, n_mc, -1).flatten(0, 1)
    return F.cosine_similarity(tf, vf, dim=1, eps=1e-8).view(B, n_mc)


def lrce_head(video_feats, text_feats, sd, task, p="fusion_model."):
    """fusionv3.py:168-198 (OE), 230-265 (MC), 360-369 (Count).
    OE/Count: video_feats (B,S,Tg,49,1024), text (B,L,768).  MC: text (B,5,L,768)."""
    B = video_feats.shape[0]
    v = _lin(video_feats, sd, p + "projection_layer.")
    v = video_pos_embed(v, sd, p + "video_pos_embed.")
    if task == "mc":
        n_mc = text_feats.shape[1]
        t = text_pos_embed(text_feats.flatten(0, 1), sd, p + "question_pos_embed.")
        v = v.unsqueeze(1).expand(-1, n_mc, -1, -1, -1).flatten(0, 1)
    else:
        t = text_pos_embed(text_feats, sd, p + "question_pos_embed.")
    s = fusion_transformer(v, t, sd)
    out = _lin(s.squeeze(), sd, p + "final_fc.")
    if task == "mc":
        return out.view(B, n_mc)
    out = out.view(B, -1)
    if task == "count":
        return F.relu(out.view(B))
    return out


def e2e_forward(sd, clips, ids, mask, types, task="oe"):
    """e2e.py:22-25 (+ MC text flattening e2e.py:77-81)."""
    vf = video_extractor(clips, sd)
    if task == "mc":
        B, n, L = ids.shape
        tf = bert(ids.flatten(0, 1), mask.flatten(0, 1), types.flatten(0, 1), sd).view(B, n, L, -1)
    else:
        tf = bert(ids, mask, types, sd)
    return lrce_head(vf, tf, sd, task)


# ----------------------------------------------------------------------------- caller (a17)
def l2_reg(params):
    """agent_base.py:103-108: sum of per-tensor L2 norms over trainable parameters."""
    r = torch.zeros((), dtype=torch.float32)
    for t in params:
        r = r + t.norm(2)
    return r


def hinge_loss(out, gt, margin):
    """agent_mc.py:20-41: mean over samples of sum_{j != gt} max(0, out_j - out_gt + margin)."""
    B, n = out.shape
    corr = out.gather(1, gt.view(-1, 1))
    h = torch.clamp(out - corr + margin, min=0)
    h = h.masked_fill(F.one_hot(gt, n).bool(), 0.0)
    return h.sum(1).mean()
