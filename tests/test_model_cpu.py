"""CPU tests of the product's host layer: state-dict schema parity with the reference (golden
fixture generated from the reference itself), constructor / argument surfaces."""
import json
import os

import pytest
import torch

from conftest import GOLDEN

CASES = {
    "msvd-qa-oe_ts3": ("oe", 1000, 32, [3]),
    "tgif-transition_ts3": ("mc", 1, 40, [3]),
    "tgif-count_ts3": ("count", 1, 30, [3]),
    "msrvtt-qa-oe_ts123": ("oe", 1500, 37, [1, 2, 3]),
}


@pytest.fixture(scope="module")
def schema():
    with open(os.path.join(GOLDEN, "state_dict_schema.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", sorted(CASES))
def test_state_dict_schema_matches_reference(schema, case):
    from lrce.models import e2e
    task, ncls, L, ts = CASES[case]
    cls = {"oe": e2e.E2EOpenEnded, "mc": e2e.E2EMultipleChoice, "count": e2e.E2ECount}[task]
    m = cls(768, ncls, 0.1, (7, 7), 1024, 5, ts, L)
    ours = {k: [list(v.shape), str(v.dtype)] for k, v in m.state_dict().items()}
    ref = schema[case]
    assert sorted(ours) == sorted(ref)
    bad = [k for k in ref if ours[k] != ref[k]]
    assert not bad, bad[:5]


def test_reference_checkpoint_extras_are_tolerated():
    """transformers 4.20 checkpoints carry bert.embeddings.position_ids (persistent buffer then)."""
    from lrce.models import e2e
    m = e2e.E2EOpenEnded(768, 1000, 0.1, (7, 7), 1024, 5, [3], 32)
    sd = m.state_dict()
    sd["text_extractor.bert.embeddings.position_ids"] = torch.arange(512).view(1, -1)
    m.load_state_dict(sd, strict=True)


def test_param_count_matches_survey():
    from lrce.models import e2e
    m = e2e.E2EOpenEnded(768, 1000, 0.1, (7, 7), 1024, 5, [3], 32)
    n = sum(p.numel() for p in m.parameters())
    assert abs(n / 1e6 - 312.2) < 0.1


def test_kinetics_backbone_checkpoint_loads(tmp_path):
    """video.py:20-26: the Swin-B Kinetics-600 checkpoint is {'state_dict': {'backbone.*', 'cls_head.*'}};
    only backbone.* (prefix stripped) goes into the extractor, strictly, via a weights_only load."""
    from lrce.feature_extractor.video import VideoExtractor
    from oracle import weights as W
    tmpl = VideoExtractor().swin.state_dict()
    filled = W.fill_state_dict({"video_extractor.swin." + k: v for k, v in tmpl.items()}, seed=3)
    ckpt = {"state_dict": {"backbone." + k[len("video_extractor.swin."):]: v for k, v in filled.items()},
            "meta": {"epoch": 30}}
    ckpt["state_dict"]["cls_head.fc_cls.weight"] = torch.zeros(600, 1024)
    path = tmp_path / "swin_base_patch244_window877_kinetics600_22k.pth"
    torch.save(ckpt, path)
    ve = VideoExtractor(str(path))
    got = ve.swin.state_dict()
    for k in ("patch_embed.proj.weight", "layers.2.blocks.17.attn.relative_position_bias_table",
              "layers.3.blocks.1.mlp.fc2.bias", "norm.weight"):
        assert torch.equal(got[k], filled["video_extractor.swin." + k]), k


@pytest.mark.parametrize("D,H,W", [(3, 25, 25), (3, 13, 13), (3, 14, 14), (3, 7, 7)])
def test_padded_window_maps_match_pad_roll_partition(D, H, W):
    """StageGeometry's window-order maps equal the reference's index movement on the padded volume:
    F.pad up to whole windows (video_swin_ori.py:253-258, padded positions = -1 here), torch.roll by
    -shift (:262), window_partition (:60-72); the inverse maps every real token to its one window row;
    the PatchMerging map pads an odd H / W (:328-331) with -1."""
    import torch.nn.functional as F
    from lrce.feature_extractor.video_swin import StageGeometry
    nc, window = 2, (8, 7, 7)
    g = StageGeometry(nc, D, H, W, window, "cpu")
    wd, wh, ww = g.ws
    idx = torch.arange(nc * D * H * W).view(nc, D, H, W)
    padded = F.pad(idx, (0, g.Wp - W, 0, g.Hp - H, 0, g.Dp - D), value=-1)

    def partition(v):
        v = v.view(nc, g.Dp // wd, wd, g.Hp // wh, wh, g.Wp // ww, ww).permute(0, 1, 3, 5, 2, 4, 6)
        return v.reshape(-1)

    assert torch.equal(g.win2sp.long(), partition(padded))
    assert g.M_win == g.win2sp.numel() and int((g.win2sp < 0).sum()) == g.M_win - g.M
    live = g.win2sp >= 0
    assert torch.equal(g.sp2win[g.win2sp[live].long()].long(), torch.nonzero(live).flatten())
    if g.shifted:
        rolled = torch.roll(padded, shifts=tuple(-s for s in g.ss), dims=(1, 2, 3))
        assert torch.equal(g.win2sp_shift.long(), partition(rolled))
    m = F.pad(idx, (0, W % 2, 0, H % 2), value=-1)
    ref = torch.stack([m[:, :, 0::2, 0::2], m[:, :, 1::2, 0::2], m[:, :, 0::2, 1::2], m[:, :, 1::2, 1::2]], -1)
    assert torch.equal(g.merge_map.long(), ref.reshape(-1))
    assert g.M_merged == nc * D * ((H + 1) // 2) * ((W + 1) // 2)


def test_gradient_freshness_claims():
    """FlatParams.claim_fresh: a weight gradient may be stored instead of accumulated only when the
    optimizer cleared the gradients and nothing has claimed that parameter since — a second backward
    before the next zero_grad accumulates, and gradients cleared any other way are never 'fresh'."""
    from lrce.flat import FlatParams
    lin = torch.nn.Linear(8, 8)
    flat = FlatParams(lin, "cpu")
    ps = [lin.weight, lin.bias]
    assert not flat.claim_fresh(ps)          # never cleared by the optimizer
    flat.grads_zeroed()
    assert flat.claim_fresh(ps)              # first writer after the clear
    assert not flat.claim_fresh(ps)          # second backward: accumulate
    assert not flat.claim_fresh([lin.weight])
    flat.grads_zeroed()
    assert flat.claim_fresh([lin.weight])
    assert not flat.claim_fresh(ps)          # the bias is fresh but the weight was claimed: accumulate


def test_decoder_kv_layer_slots():
    """The persistent decoder projects all 12 layers' memory K/V with ONE batched GEMM when the layers'
    W_kv (and biases) sit at one stride (fusionv3._layer_slots): ascending -> slot l, descending (the
    flat store's reverse forward order) -> slot n-1-l with the lowest-address layer first; anything
    else -> per-layer launches.  Checked on the real flat layout of the model and on synthetic cases."""
    from lrce.models import fusionv3 as F
    from lrce.flat import FlatParams
    from lrce.models.e2e import E2EOpenEnded

    class T:
        def __init__(self, p):
            self.p = p

        def data_ptr(self):
            return self.p
    assert F._layer_slots([T(1000 + 64 * i) for i in range(4)], 2) == ([0, 1, 2, 3], 0, 1, 32)
    assert F._layer_slots([T(1000 - 64 * i) for i in range(4)], 2) == ([3, 2, 1, 0], 3, -1, 32)
    assert F._layer_slots([T(0), T(64), T(192)], 2) is None
    assert F._layer_slots([T(0)], 2) is None
    torch.manual_seed(0)
    m = E2EOpenEnded(768, 10, 0.0, (7, 7), 1024, 5, [3], 32, swin_ckpt=None, bert_dir=None)
    flat = FlatParams(m, "cpu", order=m.lrce_param_order())   # the layout prepare() builds on the GPU
    layers = m.fusion_model.fusion_transformer.transformer.layers
    w = [flat.w16(l.multihead_attn.in_proj_weight)[768:] for l in layers]
    b = [l.multihead_attn.in_proj_bias[768:] for l in layers]
    sw, sb = F._layer_slots(w, 2), F._layer_slots(b, 4)
    assert sw is not None and sb is not None and sw[:3] == sb[:3]
    slot, first = sw[0], sw[1]
    assert sorted(slot) == list(range(12)) and slot[first] == 0


def test_overflow_guard_range_and_skip_argument():
    """FusedAdamW's found-inf guard (model.overflow_guard): BERT's encoder + embedding parameters form
    one contiguous chunk range of the flat layout, its 24 scale slots are the ones the BERT backward
    writes (one per layer and gradient, [S, 1/S, amax, found-inf]), and guard_skip clips that range to
    each update's chunk range (relative to its first chunk) or drops it."""
    from lrce.flat import FlatParams
    from lrce.models.e2e import E2EOpenEnded
    from lrce.optim import guard_skip

    slots = torch.zeros(2, 4)
    assert guard_skip(None, 0, 10) is None
    assert guard_skip(((5, 9), slots), 0, 20)[1:] == (5, 9)
    assert guard_skip(((5, 9), slots), 7, 20)[1:] == (0, 2)
    assert guard_skip(((5, 9), slots), 0, 6)[1:] == (5, 6)
    assert guard_skip(((5, 9), slots), 9, 20) is None and guard_skip(((5, 9), slots), 0, 5) is None
    torch.manual_seed(0)
    m = E2EOpenEnded(768, 10, 0.0, (7, 7), 1024, 5, [3], 32, swin_ckpt=None, bert_dir=None)
    flat = FlatParams(m, "cpu", order=m.lrce_param_order())
    params, sc = m.overflow_guard("cpu")
    assert sc.shape == (12, 2, 4) and sc is m.text_extractor.bert._grad_scales(torch.device("cpu"))
    c0, c1 = flat.chunk_range(params)                 # contiguous, or chunk_range raises
    bert = m.text_extractor.bert
    ids = {id(p) for p in params}
    assert all(id(p) in ids for p in list(bert.encoder.parameters()) + list(bert.embeddings.parameters()))
    assert not any(id(p) in ids for p in bert.pooler.parameters())
    assert c1 - c0 == sum(-(-p.numel() // 1024) for p in params)
