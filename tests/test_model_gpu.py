"""BERT, LRCE fusion and the full E2E models on the HIP path vs the reference's golden vectors and the
CPU oracle (forward and backward).  bf16 compute: tolerances relative to max|ref|."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import load_golden, csum
from helpers import load_recipe, oracle_sd, rel
from oracle import lrce_oracle as O
from oracle import weights as W

pytestmark = pytest.mark.gpu

CFG = {"msvd-qa-oe": ("oe", 1000, 32), "tgif-transition": ("mc", 1, 40), "tgif-count": ("count", 1, 30),
       "msrvtt-qa-oe": ("oe", 1500, 37)}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _bert():
    from lrce.feature_extractor.text import TextExtractor
    t = TextExtractor()
    filled = load_recipe(t, "text_extractor.")
    return t.cuda().eval(), filled


def test_bert_forward_matches_reference_golden():
    t, _ = _bert()
    g = load_golden("bert.npz")
    for sfx in ("", "2"):
        ids, mask, types = (torch.from_numpy(g[k + sfx]).cuda() for k in ("ids", "mask", "types"))
        with torch.no_grad():
            y = t(ids, mask, types)
        err = rel(y, torch.from_numpy(g["y" + sfx]))
        assert err < 5e-3, err   # fp16 forward (reference: fp16 autocast)


def test_bert_backward_matches_oracle():
    t, filled = _bert()
    g = load_golden("bert.npz")
    ids, mask, types = (torch.from_numpy(g[k]) for k in ("ids", "mask", "types"))
    R = torch.randn(ids.shape[0], ids.shape[1], 768)
    sd = oracle_sd(filled, requires_grad=True)
    yr = O.bert(ids, mask, types, sd)
    (yr * R).sum().backward()
    t.zero_grad(set_to_none=True)
    y = t(ids.cuda(), mask.cuda(), types.cuda())
    (y * R.cuda()).sum().backward()
    named = dict(t.named_parameters())
    for k in ("bert.encoder.layer.0.attention.self.query.weight", "bert.encoder.layer.11.output.dense.weight",
              "bert.encoder.layer.5.attention.output.LayerNorm.weight", "bert.encoder.layer.3.intermediate.dense.bias",
              "bert.encoder.layer.7.attention.self.value.bias", "bert.embeddings.LayerNorm.weight",
              "bert.embeddings.position_embeddings.weight", "bert.embeddings.word_embeddings.weight",
              "bert.embeddings.token_type_embeddings.weight"):
        assert rel(named[k].grad, sd["text_extractor." + k].grad) < 3e-2, k


def _fusion(task, L, ncls):
    from lrce.models.fusionv3 import LRCEOpenEnded, LRCEMultipleChoice
    cls = LRCEMultipleChoice if task == "mc" else LRCEOpenEnded
    m = cls(768, ncls, 0.1, (7, 7), 1024, 5, [3], L)
    filled = load_recipe(m, "fusion_model.")
    return m.cuda().eval(), filled


def test_fusion_oe_matches_reference_golden():
    m, _ = _fusion("oe", 32, 1000)
    g = load_golden("fusion_oe.npz")
    r = W.input_rng(int(g["seed"]))
    vf = torch.from_numpy(r.standard_normal((2, 3, 3, 49, 1024), dtype=np.float32))
    tf = torch.from_numpy(r.standard_normal((2, 32, 768), dtype=np.float32))
    with torch.no_grad():
        y = m(vf.cuda(), tf.cuda(), torch.ones(2, 32, dtype=torch.int64, device="cuda"))
    assert rel(y, torch.from_numpy(g["y"])) < 2e-2


def test_fusion_mc_matches_reference_golden():
    m, _ = _fusion("mc", 40, 1)
    g = load_golden("fusion_mc.npz")
    r = W.input_rng(int(g["seed"]))
    r.standard_normal((2, 3, 3, 49, 1024), dtype=np.float32)
    r.standard_normal((2, 32, 768), dtype=np.float32)
    vf = torch.from_numpy(r.standard_normal((1, 3, 3, 49, 1024), dtype=np.float32))
    tf = torch.from_numpy(r.standard_normal((1, 5, 40, 768), dtype=np.float32))
    np.testing.assert_allclose(csum(vf), g["vf_csum"], rtol=1e-9)
    with torch.no_grad():
        y = m(vf.cuda(), tf.cuda(), torch.ones(1, 5, 40, dtype=torch.int64, device="cuda"))
    assert rel(y, torch.from_numpy(g["y"])) < 2e-2


@pytest.mark.parametrize("task,L,ncls,B", [("oe", 32, 1000, 2), ("mc", 40, 1, 2)])
def test_fusion_backward_matches_oracle(task, L, ncls, B):
    m, filled = _fusion(task, L, ncls)
    torch.manual_seed(1)
    vf = torch.randn(B, 3, 3, 49, 1024)
    tf = torch.randn(B, 5, L, 768) if task == "mc" else torch.randn(B, L, 768)
    sd = oracle_sd(filled, requires_grad=True)
    vr, tr = vf.clone().requires_grad_(True), tf.clone().requires_grad_(True)
    yr = O.lrce_head(vr, tr, sd, task)
    R = torch.randn(yr.shape)
    (yr * R).sum().backward()
    m.zero_grad(set_to_none=True)
    vg, tg = vf.cuda().requires_grad_(True), tf.cuda().requires_grad_(True)
    y = m(vg, tg, None)
    (y * R.cuda()).sum().backward()
    assert rel(y, yr) < 2e-2
    assert rel(vg.grad, vr.grad) < 3e-2
    assert rel(tg.grad, tr.grad) < 3e-2
    named = dict(m.named_parameters())
    for k in ("fusion_transformer.transformer.layers.0.multihead_attn.in_proj_weight",
              "fusion_transformer.transformer.layers.11.multihead_attn.in_proj_bias",
              "fusion_transformer.transformer.layers.4.self_attn.in_proj_weight",
              "fusion_transformer.transformer.layers.6.self_attn.out_proj.weight",
              "fusion_transformer.transformer.layers.2.linear1.weight", "fusion_transformer.transformer.layers.9.norm3.bias",
              "fusion_transformer.summarization_token", "fusion_transformer.fusion_layer_norm.weight",
              "video_pos_embed.emb_pos", "video_pos_embed.emb_len", "video_pos_embed.emb_clip", "video_pos_embed.emb_cls",
              "question_pos_embed.emb_pos", "projection_layer.weight", "final_fc.weight", "final_fc.bias"):
        assert rel(named[k].grad, sd["fusion_model." + k].grad) < 3e-2, k


@pytest.mark.parametrize("mode", ["step", "blocks"])
@pytest.mark.parametrize("task,L,ncls,B,drop", [("oe", 32, 1000, 3, 0.1), ("oe", 32, 1000, 2, 0.0), ("mc", 40, 1, 2, 0.1),
                                                 ("mcsim", 40, 1, 2, 0.1), ("oe", 32, 1000, 12, 0.1)])
def test_fused_decoder_blocks_match_unfused(task, L, ncls, B, drop, mode, monkeypatch):
    """The fused recurrent decoder — "step": one persistent launch per recurrent step and direction
    (csrc/decoder_step.hip), "blocks": one launch per attention block (csrc/decoder.hip) — against the
    unfused launches (lrce_gemm_ln / lrce_mha / lrce_gemm) on the same inputs, in train mode with
    dropout on: all draw the same masks, so logits and every parameter / input gradient must agree to
    f32 rounding (different summation order only).  B = 12 > 10 rows: the step kernel's workgroups
    take two rows each."""
    from lrce.models.fusionv3 import LRCEOpenEnded, LRCEMultipleChoice, LRCEMultipleChoiceSim
    from lrce import kernels as K
    cls = {"oe": LRCEOpenEnded, "mc": LRCEMultipleChoice, "mcsim": LRCEMultipleChoiceSim}[task]
    torch.manual_seed(3)
    m = cls(768, ncls, drop, (7, 7), 1024, 5, [3], L).cuda().train()
    vf = torch.randn(B, 3, 3, 49, 1024, device="cuda")
    tf = torch.randn(B, 5, L, 768, device="cuda") if task != "oe" else torch.randn(B, L, 768, device="cuda")
    runs = []
    for fused in ("0", mode):
        monkeypatch.setenv("LRCE_DEC_FUSED", fused)
        m.zero_grad(set_to_none=True)
        vg, tg = vf.clone().requires_grad_(True), tf.clone().requires_grad_(True)
        torch.manual_seed(11)   # the dropout seeds the model draws
        y = m(vg, tg, None)
        R = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).cuda()
        (y.float() * R).sum().backward()
        torch.cuda.synchronize()
        assert K.dec_step_status("cuda") == 0
        runs.append((y.detach().float().clone(), vg.grad.clone(), tg.grad.clone(),
                     {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}))
    (y0, v0, t0, g0), (y1, v1, t1, g1) = runs
    assert rel(y1, y0) < 1e-4
    # the memory side (dK / dV -> bf16 -> the K/V projection's dX and dW, the embeddings) and linear1
    # (the unfused path's saved pre-activation is bf16, so dGELU sees it rounded) pass through one bf16
    # rounding: f32 differences in the last bits flip single bf16 roundings (2^-8 relative)
    assert rel(v1, v0) < 5e-3 and rel(t1, t0) < 5e-3
    assert g0.keys() == g1.keys()
    query_side = ("self_attn.", "multihead_attn.out_proj", "linear2", "norm1", "norm2", "norm3",
                  "fusion_layer_norm", "summarization_token")
    bad = {}
    for k in g0:
        err = rel(g1[k], g0[k])
        if err > (2e-4 if any(q in k for q in query_side) else 5e-3):
            bad[k] = err
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:10]


def test_step_decoder_across_row_counts(monkeypatch):
    """The persistent decoder's hand-off workspace is shared by every call on the device and re-armed
    launch by launch (the row mailboxes: the rows the previous launch wrote).  Calls with different row
    counts in sequence — 12, 5 (MC, one video), 45 (MC, nine videos: several rows per workgroup), 12 —
    must each match the unfused launches (eval mode)."""
    from lrce.models.fusionv3 import LRCEOpenEnded, LRCEMultipleChoice
    from lrce import kernels as K
    torch.manual_seed(4)
    oe = LRCEOpenEnded(768, 1000, 0.0, (7, 7), 1024, 5, [3], 32).cuda().eval()
    mc = LRCEMultipleChoice(768, 1, 0.0, (7, 7), 1024, 5, [3], 40).cuda().eval()
    cases = [(oe, 12), (mc, 1), (mc, 9), (oe, 12), (mc, 1)]
    for m, B in cases:
        vf = torch.randn(B, 3, 3, 49, 1024, device="cuda")
        tf = torch.randn(B, 5, 40, 768, device="cuda") if m is mc else torch.randn(B, 32, 768, device="cuda")
        ys = []
        for fused in ("0", "step"):
            monkeypatch.setenv("LRCE_DEC_FUSED", fused)
            with torch.no_grad():
                ys.append(m(vf, tf, None).float())
            torch.cuda.synchronize()
            assert K.dec_step_status("cuda") == 0
        assert rel(ys[1], ys[0]) < 1e-4, (B, rel(ys[1], ys[0]))


@pytest.mark.parametrize("task", ["oe", "mc"])
def test_decoder_kv_stream_is_bit_identical(task, monkeypatch):
    """The memory-side K/V projections and their input-gradient GEMMs on the "decoder_kv" stream
    (fusionv3._KV_ASYNC) run the same launches in the same order as in line: logits and every gradient
    bit-identical, in train mode with dropout on — except the video positional-embedding tables, whose
    backward adds rows with float atomics (not bit-reproducible even between two identical runs,
    tools/determinism_probe.py): those to f32 rounding."""
    from lrce.models import fusionv3 as F
    cls = {"oe": F.LRCEOpenEnded, "mc": F.LRCEMultipleChoice}[task]
    torch.manual_seed(3)
    L, B = (32, 3) if task == "oe" else (40, 2)
    m = cls(768, 1000 if task == "oe" else 1, 0.1, (7, 7), 1024, 5, [3], L).cuda().train()
    vf = torch.randn(B, 3, 3, 49, 1024, device="cuda")
    tf = torch.randn(B, L, 768, device="cuda") if task == "oe" else torch.randn(B, 5, L, 768, device="cuda")
    runs = []
    for on in (False, True):
        monkeypatch.setattr(F, "_KV_ASYNC", on)
        m.zero_grad(set_to_none=True)
        vg, tg = vf.clone().requires_grad_(True), tf.clone().requires_grad_(True)
        torch.manual_seed(11)
        y = m(vg, tg, None)
        R = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).cuda()
        (y.float() * R).sum().backward()
        torch.cuda.synchronize()
        runs.append({"y": y.detach().float().clone(), "dv": vg.grad.clone(), "dt": tg.grad.clone(),
                     **{k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}})
    assert runs[0].keys() == runs[1].keys()
    # MC: the 5 answer choices share each video row, so its dK / dV (and everything fed by it: dv, the
    # memory-side projections' gradients) accumulate by float atomics — reproducible to f32 rounding
    atomic = ("video_pos_embed.", "projection_layer.", "multihead_attn.in_proj") if task == "mc" else \
        ("video_pos_embed.",)
    # (MC: the atomically accumulated f32 dK / dV pass through a bf16 cast — a flipped rounding is 2^-8
    # of that element)
    tol = 5e-3 if task == "mc" else 1e-5
    for k in runs[0]:
        if any(a in k for a in atomic) or (task == "mc" and k == "dv"):
            assert rel(runs[1][k], runs[0][k]) < tol, k
        else:
            assert torch.equal(runs[0][k], runs[1][k]), k


def _swin_grads(ve, clips):
    ve.zero_grad(set_to_none=True)
    torch.manual_seed(7)
    y = ve(clips)
    R = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).cuda()
    (y.float() * R).sum().backward()
    torch.cuda.synchronize()
    return {k: p.grad.detach().clone() for k, p in ve.named_parameters() if p.grad is not None}


def test_swin_deferred_reductions_and_weight_gradients(monkeypatch):
    """A stage's LayerNorm gamma / beta and relative-position bias-table gradient reductions deferred to
    batched launches at the stage's first block (video_swin._DEFER_REDUCTIONS: lrce_layernorm_grad_reduce,
    lrce_wattn_dbias_batched) sum the same partials in the same order as one launch per LayerNorm /
    block: every Swin gradient bit-identical, DropPath on.  The stage's weight gradients as one
    pointer-table batched GEMM per linear (video_swin._DEFER_WGRAD, lrce_gemm_ptr_batched: one K slice
    per tile instead of split-K slabs) change only the K summation order: f32 rounding."""
    from lrce.feature_extractor import video_swin as VS
    from lrce.feature_extractor.video import VideoExtractor
    torch.manual_seed(0)
    ve = VideoExtractor(None).cuda().train()
    clips = torch.rand(1, 2, 5, 3, 224, 224, device="cuda")   # 3 x 7 x 7 windows (the bench clips)
    monkeypatch.setattr(VS, "_DEFER_WGRAD", False)
    monkeypatch.setattr(VS, "_DEFER_REDUCTIONS", False)
    g0 = _swin_grads(ve, clips)
    monkeypatch.setattr(VS, "_DEFER_REDUCTIONS", True)
    g1 = _swin_grads(ve, clips)
    monkeypatch.setattr(VS, "_DEFER_WGRAD", True)
    g2 = _swin_grads(ve, clips)
    assert g0.keys() == g1.keys() == g2.keys() and len(g0) > 0
    assert any("norm1" in k for k in g0) and any("relative_position_bias_table" in k for k in g0)
    # biases of split-K weight gradients are summed by float atomics (one add per K slice): f32 rounding
    bad = [k for k in g0 if not (rel(g1[k], g0[k]) < 1e-5 if k.endswith("bias") else torch.equal(g0[k], g1[k]))]
    assert not bad, bad[:10]
    lin = (".qkv.", ".proj.", ".fc1.", ".fc2.")
    bad = {}
    for k in g0:
        err = rel(g2[k], g0[k])
        ok = err < 1e-5 if any(t in k for t in lin) or k.endswith("bias") else torch.equal(g2[k], g0[k])
        if not ok:
            bad[k] = err
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:10]


def _e2e(name, ts=(3,)):
    from lrce.models import e2e
    task, ncls, L = CFG[name]
    cls = {"oe": e2e.E2EOpenEnded, "mc": e2e.E2EMultipleChoice, "count": e2e.E2ECount}[task]
    m = cls(768, ncls, 0.1, (7, 7), 1024, 5, list(ts), L)
    filled = load_recipe(m)
    return m.cuda().eval(), filled, task


@pytest.mark.parametrize("name,batch", [("msvd-qa-oe", 2), ("tgif-transition", 1), ("tgif-count", 2),
                                        ("msrvtt-qa-oe", 1)])
def test_e2e_logits_match_reference_golden(name, batch):
    g = load_golden(f"e2e_{name}_b{batch}.npz")
    ts = tuple(int(x) for x in g["temporal_scale"])
    m, filled, task = _e2e(name, ts)
    clips = W.synthetic_clips(batch, sum(ts), seed=int(g["seed"]))
    np.testing.assert_allclose(csum(clips), g["clips_csum"], rtol=1e-9)
    with torch.no_grad():
        y = m(clips.cuda(), *(torch.from_numpy(g[k]).cuda() for k in ("ids", "mask", "types")))
    ref = torch.from_numpy(g["logits"])
    assert y.shape == ref.shape
    # BASELINE north_star bar "1e-2 bf16", relative to max|logit|, for every head (no per-head
    # escape hatch).  The BERT forward runs in fp16 like the reference's fp16 autocast; Swin and
    # the decoder memory path in bf16, the decoder query side in exact f32.
    err = rel(y, ref)
    assert err < 1e-2, (name, err)


@pytest.mark.parametrize("name,batch", [("msvd-qa-oe", 10), ("msrvtt-qa-oe", 10), ("tgif-transition", 9)])
def test_baseline_config_forward_matches_oracle(name, batch):
    """BASELINE.json configs 2-5 at their own batch sizes (bs 10 msvd / msrvtt with temporal scale 3,
    bs 9 tgif-transition 5-way MC; reference shapes e2e.py:22-25, fusionv3.py:230-265): eval-mode
    logits of the HIP path vs the fp32 CPU oracle on the same synthetic batch, within the north-star
    1e-2 (relative to max|logit|).  These are the tile / split choices the bench runs at bs 10."""
    m, filled, task = _e2e(name, (3,))
    L = CFG[name][2]
    clips = W.synthetic_clips(batch, 3, seed=21)
    if task == "mc":
        ids, mask, types = W.synthetic_question(batch, L, seed=21, n_choice=5, ans_tokens=8)
    else:
        ids, mask, types = W.synthetic_question(batch, L, seed=21)
    with torch.no_grad():
        y = m(clips.cuda(), ids.cuda(), mask.cuda(), types.cuda()).float().cpu()
    del m
    torch.set_num_threads(min(16, torch.get_num_threads()))
    with torch.no_grad():
        yr = O.e2e_forward(oracle_sd(filled), clips, ids, mask, types, task)
    assert y.shape == yr.shape
    err = rel(y, yr)
    assert err < 1e-2, (name, batch, err)


def test_e2e_train_step_grads_match_oracle():
    """Full model, CE + L2 loss (agent_oe.py:35-36), dropout off: parameter grads vs oracle autograd."""
    m, filled, _ = _e2e("msvd-qa-oe")
    clips = W.synthetic_clips(1, 3, seed=9)
    ids, mask, types = W.synthetic_question(1, 32, seed=9)
    label = torch.tensor([17])
    sd = oracle_sd(filled, requires_grad=True)
    yr = O.e2e_forward(sd, clips, ids, mask, types, "oe")
    F.cross_entropy(yr, label).backward()
    m.zero_grad(set_to_none=True)
    y = m(clips.cuda(), ids.cuda(), mask.cuda(), types.cuda())
    F.cross_entropy(y, label.cuda()).backward()
    named = dict(m.named_parameters())
    worst = {}
    for k in ("video_extractor.swin.patch_embed.proj.weight", "video_extractor.swin.patch_embed.proj.bias",
              "video_extractor.swin.patch_embed.norm.weight", "video_extractor.swin.layers.0.blocks.1.attn.qkv.weight",
              "video_extractor.swin.layers.2.blocks.17.mlp.fc2.weight",
              "video_extractor.swin.layers.1.blocks.0.attn.relative_position_bias_table",
              "video_extractor.swin.layers.3.blocks.1.norm2.weight", "video_extractor.swin.norm.weight",
              "text_extractor.bert.encoder.layer.0.attention.self.key.weight",
              "fusion_model.fusion_transformer.transformer.layers.0.linear2.weight", "fusion_model.final_fc.weight"):
        worst[k] = rel(named[k].grad, sd[k].grad)
    assert max(worst.values()) < 5e-2, worst


def _mcsim_inputs(g):
    r = W.input_rng(int(g["seed"]))
    vf = torch.from_numpy(r.standard_normal((2, 3, 3, 49, 1024), dtype=np.float32))
    tf = torch.from_numpy(r.standard_normal((2, 5, 40, 768), dtype=np.float32))
    return vf, tf


def test_fusion_mc_sim_matches_reference_golden_and_oracle_grads():
    """LRCEMultipleChoiceSim (fusionv3.py:268-333): FusionVideo (video-only memory) on the native
    recurrent decoder + text projection + cosine.  Outputs vs the reference's golden (the cosines
    are ~0.05 in size: tolerance is absolute, 1e-3, as for fp32 logits); gradients vs the oracle."""
    from lrce.models.fusionv3 import LRCEMultipleChoiceSim
    m = LRCEMultipleChoiceSim(768, 1, 0.1, (7, 7), 1024, 5, [3], 40)
    filled = load_recipe(m, "fusion_model.")
    m = m.cuda().eval()
    g = load_golden("fusion_mcsim.npz")
    vf, tf = _mcsim_inputs(g)
    mask = torch.ones(2, 5, 40, dtype=torch.int64, device="cuda")
    with torch.no_grad():
        y = m(vf.cuda(), tf.cuda(), mask).float().cpu()
    assert float((y - torch.from_numpy(g["y"])).abs().max()) < 1e-3
    # backward (eval mode, deterministic) vs the oracle's autograd
    R = torch.randn(2, 5)
    sd = oracle_sd(filled, requires_grad=True)
    (O.lrce_mc_sim(vf, tf, sd) * R).sum().backward()
    out = m(vf.cuda(), tf.cuda(), mask)
    (out * R.cuda()).sum().backward()
    named = dict(m.named_parameters())
    for k in ("text_projection.weight", "text_projection.bias", "fusion_transformer.summarization_token",
              "fusion_transformer.transformer.layers.11.linear2.weight",
              "fusion_transformer.transformer.layers.0.multihead_attn.in_proj_weight",
              "video_pos_embed.emb_pos", "question_pos_embed.emb_pos", "projection_layer.weight"):
        assert rel(named[k].grad, sd["fusion_model." + k].grad) < 5e-2, k
