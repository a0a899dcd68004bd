"""Pin the CPU oracle (oracle/lrce_oracle.py) against golden vectors produced by running the
reference implementation itself (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import csum, load_golden
from oracle import lrce_oracle as O
from oracle import weights as W


class RecipeSD(dict):
    """Lazily materialised recipe state dict: sd[key] -> weight from oracle/weights.py."""

    def __missing__(self, key):
        if key.endswith("relative_position_bias_table"):
            nH = {"layers.0": 4, "layers.1": 8, "layers.2": 16, "layers.3": 32}[key.split("swin.")[1][:8]]
            shape = (2535, nH)
        else:
            shape = SHAPES[key]
        v = W.value_for(key, shape)
        self[key] = v
        return v


def _swin_shapes():
    s = {}
    p = "video_extractor.swin."
    s[p + "patch_embed.proj.weight"] = (128, 3, 2, 4, 4)
    s[p + "patch_embed.proj.bias"] = (128,)
    s[p + "patch_embed.norm.weight"] = (128,)
    s[p + "patch_embed.norm.bias"] = (128,)
    for i, (dep, C) in enumerate(zip((2, 2, 18, 2), (128, 256, 512, 1024))):
        for b in range(dep):
            q = f"{p}layers.{i}.blocks.{b}."
            for n in ("norm1", "norm2"):
                s[q + n + ".weight"] = (C,)
                s[q + n + ".bias"] = (C,)
            s[q + "attn.qkv.weight"] = (3 * C, C)
            s[q + "attn.qkv.bias"] = (3 * C,)
            s[q + "attn.proj.weight"] = (C, C)
            s[q + "attn.proj.bias"] = (C,)
            s[q + "mlp.fc1.weight"] = (4 * C, C)
            s[q + "mlp.fc1.bias"] = (4 * C,)
            s[q + "mlp.fc2.weight"] = (C, 4 * C)
            s[q + "mlp.fc2.bias"] = (C,)
        if i < 3:
            s[f"{p}layers.{i}.downsample.norm.weight"] = (4 * C,)
            s[f"{p}layers.{i}.downsample.norm.bias"] = (4 * C,)
            s[f"{p}layers.{i}.downsample.reduction.weight"] = (2 * C, 4 * C)
    s[p + "norm.weight"] = (1024,)
    s[p + "norm.bias"] = (1024,)
    return s


def _bert_shapes():
    s = {}
    p = "text_extractor.bert."
    s[p + "embeddings.word_embeddings.weight"] = (30522, 768)
    s[p + "embeddings.position_embeddings.weight"] = (512, 768)
    s[p + "embeddings.token_type_embeddings.weight"] = (2, 768)
    s[p + "embeddings.LayerNorm.weight"] = (768,)
    s[p + "embeddings.LayerNorm.bias"] = (768,)
    for i in range(12):
        q = f"{p}encoder.layer.{i}."
        for n in ("attention.self.query", "attention.self.key", "attention.self.value", "attention.output.dense"):
            s[q + n + ".weight"] = (768, 768)
            s[q + n + ".bias"] = (768,)
        s[q + "intermediate.dense.weight"] = (3072, 768)
        s[q + "intermediate.dense.bias"] = (3072,)
        s[q + "output.dense.weight"] = (768, 3072)
        s[q + "output.dense.bias"] = (768,)
        for n in ("attention.output.LayerNorm", "output.LayerNorm"):
            s[q + n + ".weight"] = (768,)
            s[q + n + ".bias"] = (768,)
    return s


def fusion_shapes(L, S, num_classes, prefix="fusion_model."):
    s = {}
    p = prefix
    s[p + "video_pos_embed.emb_cls"] = (1, 1, 1, 1, 768)
    s[p + "video_pos_embed.emb_pos"] = (1, 1, 1, 50, 768)
    s[p + "video_pos_embed.emb_len"] = (1, 1, 3, 1, 768)
    s[p + "video_pos_embed.emb_clip"] = (1, S, 1, 1, 768)
    s[p + "question_pos_embed.emb_cls"] = (1, 1, 768)
    s[p + "question_pos_embed.emb_pos"] = (1, L + 1, 768)
    for n in ("video_pos_embed.layer_norm", "question_pos_embed.layer_norm", "fusion_transformer.fusion_layer_norm"):
        s[p + n + ".weight"] = (768,)
        s[p + n + ".bias"] = (768,)
    s[p + "projection_layer.weight"] = (768, 1024)
    s[p + "projection_layer.bias"] = (768,)
    s[p + "fusion_transformer.summarization_token"] = (1, 1, 768)
    for k in range(12):
        q = f"{p}fusion_transformer.transformer.layers.{k}."
        for a in ("self_attn", "multihead_attn"):
            s[q + a + ".in_proj_weight"] = (2304, 768)
            s[q + a + ".in_proj_bias"] = (2304,)
            s[q + a + ".out_proj.weight"] = (768, 768)
            s[q + a + ".out_proj.bias"] = (768,)
        s[q + "linear1.weight"] = (3072, 768)
        s[q + "linear1.bias"] = (3072,)
        s[q + "linear2.weight"] = (768, 3072)
        s[q + "linear2.bias"] = (768,)
        for n in ("norm1", "norm2", "norm3"):
            s[q + n + ".weight"] = (768,)
            s[q + n + ".bias"] = (768,)
    s[p + "final_fc.weight"] = (num_classes, 768)
    s[p + "final_fc.bias"] = (num_classes,)
    return s


SHAPES = {}
SHAPES.update(_swin_shapes())
SHAPES.update(_bert_shapes())


def recipe_sd(L=32, S=3, num_classes=1000):
    SHAPES.update(fusion_shapes(L, S, num_classes))
    return RecipeSD()


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max())


def test_relative_position_index_slice_is_subwindow():
    """index[:147,:147] of the 8x7x7 table == the 3x7x7 window's own index."""
    full = O.relative_position_index((8, 7, 7))[:147, :147]
    g = torch.stack(torch.meshgrid(torch.arange(3), torch.arange(7), torch.arange(7), indexing="ij")).flatten(1)
    rel_ = (g[:, :, None] - g[:, None, :]).permute(1, 2, 0) + torch.tensor([7, 6, 6])
    own = rel_[..., 0] * 169 + rel_[..., 1] * 13 + rel_[..., 2]
    assert torch.equal(full, own)


def test_patch_embed_golden():
    g = load_golden("patch_embed.npz")
    r = W.input_rng(int(g["seed"]))
    x = torch.from_numpy(r.standard_normal((2, 3, 5, 32, 48), dtype=np.float32))
    np.testing.assert_allclose(csum(x), g["x_csum"], rtol=1e-9)
    sd = recipe_sd()
    y = O.patch_embed(x, sd, "video_extractor.swin.patch_embed.").permute(0, 4, 1, 2, 3)
    assert rel(y, torch.from_numpy(g["y"])) < 1e-5


@pytest.mark.parametrize("tag", ["stage1_28", "stage3_14", "stage4_7"])
def test_swin_stage_golden(tag):
    g = load_golden(f"swin_{tag}.npz")
    dim, heads, hw, st = int(g["dim"]), int(g["heads"]), int(g["hw"]), int(g["stage"])
    r = W.input_rng(int(g["seed"]))
    x = torch.from_numpy(r.standard_normal((1, dim, 3, hw, hw), dtype=np.float32))
    np.testing.assert_allclose(csum(x), g["x_csum"], rtol=1e-9)
    sd = recipe_sd()
    y = O.swin_stage(x.permute(0, 2, 3, 4, 1), sd, f"video_extractor.swin.layers.{st}.", 2, heads,
                     bool(g["downsample"])).permute(0, 4, 1, 2, 3)
    assert rel(y, torch.from_numpy(g["y"])) < 1e-5


def test_bert_golden():
    g = load_golden("bert.npz")
    sd = recipe_sd()
    for sfx in ("", "2"):
        y = O.bert(torch.from_numpy(g["ids" + sfx]), torch.from_numpy(g["mask" + sfx]),
                   torch.from_numpy(g["types" + sfx]), sd)
        assert rel(y, torch.from_numpy(g["y" + sfx])) < 1e-5


def test_fusion_oe_golden():
    g = load_golden("fusion_oe.npz")
    r = W.input_rng(int(g["seed"]))
    vf = torch.from_numpy(r.standard_normal((2, 3, 3, 49, 1024), dtype=np.float32))
    tf = torch.from_numpy(r.standard_normal((2, 32, 768), dtype=np.float32))
    np.testing.assert_allclose(csum(vf), g["vf_csum"], rtol=1e-9)
    sd = recipe_sd(32, 3, 1000)
    y = O.lrce_head(vf, tf, sd, "oe")
    assert rel(y, torch.from_numpy(g["y"])) < 1e-5


def test_fusion_mc_golden():
    g = load_golden("fusion_mc.npz")
    r = W.input_rng(int(g["seed"]))
    r.standard_normal((2, 3, 3, 49, 1024), dtype=np.float32)
    r.standard_normal((2, 32, 768), dtype=np.float32)
    vf = torch.from_numpy(r.standard_normal((1, 3, 3, 49, 1024), dtype=np.float32))
    tf = torch.from_numpy(r.standard_normal((1, 5, 40, 768), dtype=np.float32))
    np.testing.assert_allclose(csum(vf), g["vf_csum"], rtol=1e-9)
    sd = recipe_sd(40, 3, 1)
    y = O.lrce_head(vf, tf, sd, "mc")
    assert rel(y, torch.from_numpy(g["y"])) < 1e-5


def test_hinge_loss_matches_reference_loop():
    """agent_mc.py:20-41 restated as a loop here vs the vectorised oracle."""
    g = torch.Generator().manual_seed(0)
    out = torch.randn(6, 5, generator=g)
    gt = torch.randint(0, 5, (6,), generator=g)
    ref = []
    for i in range(6):
        c = int(gt[i])
        terms = [max(0.0, float(out[i, j] - out[i, c]) + 1.0) for j in range(5) if j != c]
        ref.append(sum(terms))
    assert abs(float(O.hinge_loss(out, gt, 1.0)) - sum(ref) / 6) < 1e-6


@pytest.mark.slow
@pytest.mark.parametrize("name,task,L,ncls", [("msvd-qa-oe_b2", "oe", 32, 1000),
                                              ("tgif-transition_b1", "mc", 40, 1),
                                              ("tgif-count_b2", "count", 30, 1)])
def test_e2e_golden(name, task, L, ncls):
    g = load_golden(f"e2e_{name}.npz")
    B = int(g["batch"])
    S = int(np.sum(g["temporal_scale"]))
    clips = W.synthetic_clips(B, S, seed=int(g["seed"]))
    np.testing.assert_allclose(csum(clips), g["clips_csum"], rtol=1e-9)
    sd = recipe_sd(L, S, ncls)
    with torch.no_grad():
        y = O.e2e_forward(sd, clips, torch.from_numpy(g["ids"]), torch.from_numpy(g["mask"]),
                          torch.from_numpy(g["types"]), task)
    assert rel(y, torch.from_numpy(g["logits"])) < 1e-4


def test_pil_bilinear_restatement_matches_pillow_fixture():
    """oracle/video_resize.py (Pillow's fixed-point antialiased bilinear) == Pillow 12.2.0's output."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_video_golden import CASES, frames_for
    from oracle.video_resize import pil_bilinear_resize
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "frames_resize.npz"))
    for name, n, h, w, pick, oh, ow in CASES:
        fr = frames_for(name, n, h, w)
        assert np.array_equal(pil_bilinear_resize(fr[pick], oh, ow), g[name]), name


def test_multiscale_indices_restatement():
    """16 frames, 5 per clip, scale 3 -> frames 0-4, 5-9, 10-14; product == oracle."""
    from oracle.video_resize import multiscale_frame_indices as ref
    from lrce.dataset.video import multiscale_frame_indices as ours, extracted_scale_index
    assert ref(16, 5, [3]) == list(range(15))
    for T in (5, 6, 9, 16, 17, 40, 121, 300):
        for ts in ([1], [2], [3], [1, 2, 3], [3, 1]):
            try:
                r = ref(T, 5, ts)
            except AssertionError:
                with pytest.raises(ValueError):
                    ours(T, 5, ts)
                continue
            assert ours(T, 5, ts) == r, (T, ts)
    assert extracted_scale_index([1, 2, 3]) == [0, 1, 2, 3, 4, 5] and extracted_scale_index([3]) == [3, 4, 5]


def test_mc_sim_oracle_matches_reference_golden():
    """LRCEMultipleChoiceSim (fusionv3.py:268-333): oracle vs the reference's own output; our module's
    state-dict keys == the reference's (text_projection added, no final_fc)."""
    from lrce.models.fusionv3 import LRCEMultipleChoiceSim
    g = load_golden("fusion_mcsim.npz")
    m = LRCEMultipleChoiceSim(768, 1, 0.1, (7, 7), 1024, 5, [3], 40)
    assert sorted(m.state_dict()) == [str(k) for k in g["keys"]]
    sd = W.fill_state_dict({"fusion_model." + k: v for k, v in m.state_dict().items()})
    r = W.input_rng(int(g["seed"]))
    vf = torch.from_numpy(r.standard_normal((2, 3, 3, 49, 1024), dtype=np.float32))
    tf = torch.from_numpy(r.standard_normal((2, 5, 40, 768), dtype=np.float32))
    np.testing.assert_allclose(csum(vf), g["vf_csum"], rtol=1e-9)
    with torch.no_grad():
        y = O.lrce_mc_sim(vf, tf, sd)
    assert float((y - torch.from_numpy(g["y"])).abs().max()) < 1e-5
