"""Generate golden vectors by running the REFERENCE implementation (/root/reference, read-only)
on deterministic inputs and the deterministic weight recipe (oracle/weights.py).

Run in the survey container only (the reference does not exist on the GPU box):
    python tests/golden/make_golden.py
Outputs tests/golden/*.npz (inputs that are cheap to regenerate are stored as seeds + a
checksum; outputs are stored in full or as fixed slices).  The script imports reference modules
as libraries; nothing from the reference is copied into this repository.
"""
import contextlib
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import refstubs  # noqa: E402

refstubs.install()

import transformers  # noqa: E402
from oracle import weights as W  # noqa: E402

torch.set_grad_enabled(False)
torch.set_num_threads(os.cpu_count())

CONFIGS = {  # /root/reference/configs/*.json
    "msvd-qa-oe": dict(text_seq_len=32, num_classes=1000, task="oe"),
    "msrvtt-qa-oe": dict(text_seq_len=37, num_classes=1500, task="oe"),
    "tgif-transition": dict(text_seq_len=40, num_classes=1, task="mc"),
    "tgif-count": dict(text_seq_len=30, num_classes=1, task="count"),
}


def fill(module, prefix=""):
    sd = module.state_dict()
    full = {prefix + k: v for k, v in sd.items()}
    filled = W.fill_state_dict(full)
    module.load_state_dict({k[len(prefix):]: v for k, v in filled.items()}, strict=True)
    return module


@contextlib.contextmanager
def reference_model_env():
    """E2EBase asserts a checkpoint path relative to cwd and calls torch.load /
    BertModel.from_pretrained (network).  Serve both from the weight recipe instead."""
    from lrce.feature_extractor import video as ref_video
    from lrce.feature_extractor.video_swin_ori import SwinTransformer3D

    tmpl = SwinTransformer3D(embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32], patch_size=(2, 4, 4),
                             window_size=(8, 7, 7), drop_path_rate=0.2, patch_norm=True).state_dict()
    swin_sd = W.fill_state_dict({"video_extractor.swin." + k: v for k, v in tmpl.items()})
    ckpt = {"state_dict": {"backbone." + k[len("video_extractor.swin."):]: v for k, v in swin_sd.items()}}
    old_load = ref_video.torch.load
    old_fp = transformers.BertModel.from_pretrained
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, "pretrained_models"))
        open(os.path.join(td, "pretrained_models", "swin_base_patch244_window877_kinetics600_22k.pth"), "w").close()
        os.chdir(td)
        ref_video.torch.load = lambda *a, **k: ckpt
        transformers.BertModel.from_pretrained = classmethod(lambda cls, *a, **k: transformers.BertModel(transformers.BertConfig()))
        try:
            yield
        finally:
            ref_video.torch.load = old_load
            transformers.BertModel.from_pretrained = old_fp
            os.chdir(cwd)


def build_e2e(cfg, temporal_scale=(3,)):
    from lrce.models import e2e
    cls = {"oe": e2e.E2EOpenEnded, "mc": e2e.E2EMultipleChoice, "count": e2e.E2ECount}[cfg["task"]]
    with reference_model_env():
        m = cls(768, cfg["num_classes"], 0.1, (7, 7), 1024, 5, list(temporal_scale), cfg["text_seq_len"])
    fill(m)
    m.eval()
    m.video_extractor.swin.eval()
    return m


def csum(t):
    t = t.double()
    return np.array([t.sum().item(), (t * t).sum().item(), t.abs().max().item()])


def full_model(name, batch, seed, ts=(3,)):
    cfg = CONFIGS[name]
    m = build_e2e(cfg, ts)
    S = sum(ts)
    clips = W.synthetic_clips(batch, S, seed=seed)
    if cfg["task"] == "mc":
        ids, mask, types = W.synthetic_question(batch, cfg["text_seq_len"], seed=seed, n_choice=5, ans_tokens=6)
    else:
        ids, mask, types = W.synthetic_question(batch, cfg["text_seq_len"], seed=seed)
    vf = m.extract_video_features(clips)
    tf = m.extract_text_features(ids, mask, types)
    logits = m.fusion_model(vf, tf, mask)
    logits2 = m(clips, ids, mask, types)
    assert torch.equal(logits, logits2)
    out = dict(clips_csum=csum(clips), ids=ids.numpy(), mask=mask.numpy(), types=types.numpy(),
               video_features_slice=vf[..., :64].numpy(), video_features_csum=csum(vf),
               text_features=tf.numpy(), logits=logits.numpy(), batch=batch, seed=seed,
               temporal_scale=np.array(ts))
    np.savez_compressed(os.path.join(HERE, f"e2e_{name}_b{batch}.npz"), **out)
    print(name, "logits", logits.flatten()[:6].tolist())


def swin_stage_fixture(tag, stage, dim, heads, hw, downsample, seed):
    from lrce.feature_extractor.video_swin_ori import BasicLayer, PatchMerging
    layer = BasicLayer(dim=dim, depth=2, num_heads=heads, window_size=(8, 7, 7), drop_path=[0.0, 0.0], qkv_bias=True,
                       downsample=PatchMerging if downsample else None)
    fill(layer, f"video_extractor.swin.layers.{stage}.")
    layer.eval()
    r = W.input_rng(seed)
    x = torch.from_numpy(r.standard_normal((1, dim, 3, hw, hw), dtype=np.float32))
    y = layer(x)
    np.savez_compressed(os.path.join(HERE, f"swin_{tag}.npz"), x_csum=csum(x), y=y.numpy(), seed=seed, hw=hw, stage=stage,
                        dim=dim, heads=heads, downsample=downsample)
    print(tag, tuple(y.shape))


def patch_embed_fixture(seed):
    from lrce.feature_extractor.video_swin_ori import PatchEmbed3D
    pe = PatchEmbed3D(patch_size=(2, 4, 4), in_chans=3, embed_dim=128, norm_layer=torch.nn.LayerNorm)
    fill(pe, "video_extractor.swin.patch_embed.")
    r = W.input_rng(seed)
    x = torch.from_numpy(r.standard_normal((2, 3, 5, 32, 48), dtype=np.float32))
    y = pe(x)
    np.savez_compressed(os.path.join(HERE, "patch_embed.npz"), x_csum=csum(x), y=y.numpy(), seed=seed)


def fusion_fixture(seed):
    from lrce.models.fusionv3 import LRCEOpenEnded, LRCEMultipleChoice
    r = W.input_rng(seed)
    m = LRCEOpenEnded(768, 1000, 0.1, (7, 7), 1024, 5, [3], 32)
    fill(m, "fusion_model.")
    m.eval()
    vf = torch.from_numpy(r.standard_normal((2, 3, 3, 49, 1024), dtype=np.float32))
    tf = torch.from_numpy(r.standard_normal((2, 32, 768), dtype=np.float32))
    mask = torch.ones(2, 32, dtype=torch.int64)
    y = m(vf, tf, mask)
    summ = m.fusion_transformer(m.video_pos_embed(m.projection_layer(vf)), m.question_pos_embed(tf), mask)
    np.savez_compressed(os.path.join(HERE, "fusion_oe.npz"), vf_csum=csum(vf), tf_csum=csum(tf), y=y.numpy(), seed=seed,
                        summ=summ.numpy())
    mc = LRCEMultipleChoice(768, 1, 0.1, (7, 7), 1024, 5, [3], 40)
    fill(mc, "fusion_model.")
    mc.eval()
    vf1 = torch.from_numpy(r.standard_normal((1, 3, 3, 49, 1024), dtype=np.float32))
    tf1 = torch.from_numpy(r.standard_normal((1, 5, 40, 768), dtype=np.float32))
    y1 = mc(vf1, tf1, torch.ones(1, 5, 40, dtype=torch.int64))
    np.savez_compressed(os.path.join(HERE, "fusion_mc.npz"), vf_csum=csum(vf1), tf_csum=csum(tf1), y=y1.numpy(), seed=seed)


def fusion_mcsim_fixture(seed):
    """LRCEMultipleChoiceSim (fusionv3.py:268-333): FusionVideo + text projection + cosine."""
    from lrce.models.fusionv3 import LRCEMultipleChoiceSim
    r = W.input_rng(seed)
    m = LRCEMultipleChoiceSim(768, 1, 0.1, (7, 7), 1024, 5, [3], 40)
    fill(m, "fusion_model.")
    m.eval()
    vf = torch.from_numpy(r.standard_normal((2, 3, 3, 49, 1024), dtype=np.float32))
    tf = torch.from_numpy(r.standard_normal((2, 5, 40, 768), dtype=np.float32))
    y = m(vf, tf, torch.ones(2, 5, 40, dtype=torch.int64))
    keys = sorted(m.state_dict())
    np.savez_compressed(os.path.join(HERE, "fusion_mcsim.npz"), vf_csum=csum(vf), tf_csum=csum(tf), y=y.numpy(),
                        seed=seed, keys=np.array(keys))


def bert_fixture(seed):
    b = transformers.BertModel(transformers.BertConfig())
    fill(b, "text_extractor.bert.")
    b.eval()
    ids, mask, types = W.synthetic_question(3, 32, seed=seed)
    mask[2, 25:] = 0
    ids2, mask2, types2 = W.synthetic_question(2, 40, seed=seed + 1, n_choice=None, ans_tokens=6)
    y = b(input_ids=ids, attention_mask=mask, token_type_ids=types).last_hidden_state
    y2 = b(input_ids=ids2, attention_mask=mask2, token_type_ids=types2).last_hidden_state
    np.savez_compressed(os.path.join(HERE, "bert.npz"), ids=ids.numpy(), mask=mask.numpy(), types=types.numpy(),
                        y=y.numpy(), ids2=ids2.numpy(), mask2=mask2.numpy(), types2=types2.numpy(), y2=y2.numpy())


def schema_fixture():
    """State-dict key schema (name -> shape, dtype) of the reference E2E models: the drop-in contract
    for checkpoints."""
    import json
    out = {}
    for name, ts in (("msvd-qa-oe", (3,)), ("tgif-transition", (3,)), ("tgif-count", (3,)), ("msrvtt-qa-oe", (1, 2, 3))):
        m = build_e2e(CONFIGS[name], ts)
        out[f"{name}_ts{''.join(map(str, ts))}"] = {k: [list(v.shape), str(v.dtype)] for k, v in m.state_dict().items()}
    with open(os.path.join(HERE, "state_dict_schema.json"), "w") as f:
        json.dump(out, f, sort_keys=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["ops", "e2e", "schema"]
    if "schema" in which:
        schema_fixture()
    if "ops" in which:
        patch_embed_fixture(11)
        swin_stage_fixture("stage1_28", 0, 128, 4, 28, True, 12)
        swin_stage_fixture("stage3_14", 2, 512, 16, 14, True, 13)
        swin_stage_fixture("stage4_7", 3, 1024, 32, 7, False, 14)
        bert_fixture(15)
        fusion_fixture(16)
    if "mcsim" in which or "ops" in which:
        fusion_mcsim_fixture(17)
    if "e2e" in which:
        full_model("msvd-qa-oe", 2, 1)
        full_model("tgif-transition", 1, 2)
        full_model("tgif-count", 2, 3)
        full_model("msrvtt-qa-oe", 1, 4, ts=(1, 2))
