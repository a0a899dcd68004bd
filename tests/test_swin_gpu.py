"""Video Swin-B 3D on the HIP path vs the reference's golden vectors and the CPU oracle (fwd + bwd).
bf16 compute: tolerances are relative to max|ref| (BASELINE.json north_star: 1e-2 bf16)."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from helpers import load_recipe, oracle_sd, rel
from oracle import lrce_oracle as O
from oracle import weights as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def swin():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lrce.feature_extractor.video import VideoExtractor
    v = VideoExtractor()
    filled = load_recipe(v, "video_extractor.")
    v = v.cuda().eval()
    return v, filled


@pytest.mark.parametrize("tag", ["stage1_28", "stage3_14", "stage4_7"])
def test_stage_matches_reference_golden(swin, tag):
    v, _ = swin
    g = load_golden(f"swin_{tag}.npz")
    dim, hw, st = int(g["dim"]), int(g["hw"]), int(g["stage"])
    r = W.input_rng(int(g["seed"]))
    x = torch.from_numpy(r.standard_normal((1, dim, 3, hw, hw), dtype=np.float32))
    with torch.no_grad():
        y = v.swin.forward_stage(st, x.permute(0, 2, 3, 4, 1).contiguous().cuda(), depth=2)
    ref = torch.from_numpy(g["y"]).permute(0, 2, 3, 4, 1)
    assert rel(y, ref) < 1e-2


def test_stage_backward_matches_oracle(swin):
    v, filled = swin
    torch.manual_seed(0)
    x = torch.randn(2, 3, 14, 14, 512)
    R = torch.randn(2, 3, 7, 7, 1024)
    sd = oracle_sd(filled, requires_grad=True)
    xr = x.clone().requires_grad_(True)
    yr = O.swin_stage(xr, sd, "video_extractor.swin.layers.2.", 2, 16, True)
    (yr * R).sum().backward()
    v.zero_grad(set_to_none=True)
    xg = x.cuda().requires_grad_(True)
    y = v.swin.forward_stage(2, xg, depth=2)
    (y * R.cuda()).sum().backward()
    assert rel(y, yr) < 1e-2
    assert rel(xg.grad, xr.grad) < 2e-2
    p = "video_extractor.swin.layers.2."
    named = dict(v.named_parameters())
    for k in ("blocks.0.attn.qkv.weight", "blocks.1.attn.qkv.bias", "blocks.1.attn.relative_position_bias_table",
              "blocks.0.norm1.weight", "blocks.1.norm2.bias", "blocks.0.mlp.fc1.weight", "blocks.1.mlp.fc2.weight",
              "blocks.1.mlp.fc2.bias", "blocks.0.attn.proj.weight", "downsample.reduction.weight",
              "downsample.norm.weight"):
        got = named["swin.layers.2." + k].grad
        assert rel(got, sd[p + k].grad) < 3e-2, k


@pytest.mark.parametrize("stage,hw", [(1, 25), (2, 13)])
def test_padded_stage_matches_oracle(swin, stage, hw):
    """Volumes that are not whole windows: the reference zero-pads norm1's output up to the window
    (video_swin_ori.py:253-258), builds the shift mask over the padded volume (:346) and crops after
    the attention; PatchMerging pads an odd H / W before its 2x2 gather (:328-331).  Stage 2 at 25x25
    (padded to 28, odd merge) and stage 3 at 13x13 (padded to 14) against the oracle, which restates
    those lines (parity at these sizes is pinned by the oracle's restatement; the reference golden
    vectors cover whole-window sizes)."""
    v, filled = swin
    dim, nH = (256, 8) if stage == 1 else (512, 16)
    torch.manual_seed(1)
    x = torch.randn(2, 3, hw, hw, dim)
    m = (hw + 1) // 2
    R = torch.randn(2, 3, m, m, 2 * dim)
    sd = oracle_sd(filled, requires_grad=True)
    p = f"video_extractor.swin.layers.{stage}."
    xr = x.clone().requires_grad_(True)
    yr = O.swin_stage(xr, sd, p, 2, nH, True)
    (yr * R).sum().backward()
    v.zero_grad(set_to_none=True)
    xg = x.cuda().requires_grad_(True)
    y = v.swin.forward_stage(stage, xg, depth=2)
    (y * R.cuda()).sum().backward()
    assert y.shape == yr.shape
    assert rel(y, yr) < 1e-2
    assert rel(xg.grad, xr.grad) < 2e-2
    named = dict(v.named_parameters())
    for k in ("blocks.0.attn.qkv.weight", "blocks.1.attn.relative_position_bias_table", "blocks.0.norm1.weight",
              "blocks.0.norm1.bias", "blocks.1.norm1.bias", "blocks.1.mlp.fc1.weight", "downsample.norm.weight",
              "downsample.norm.bias", "downsample.reduction.weight"):
        assert rel(named[f"swin.layers.{stage}." + k].grad, sd[p + k].grad) < 3e-2, k


def test_video_extractor_matches_oracle(swin):
    v, filled = swin
    clips = W.synthetic_clips(1, 3, seed=5)
    with torch.no_grad():
        f = v(clips.cuda())
        fr = O.video_extractor(clips, oracle_sd(filled))
    assert f.shape == (1, 3, 3, 49, 1024)
    assert rel(f, fr) < 2e-2


def test_video_extractor_matches_golden_slice(swin):
    v, _ = swin
    g = load_golden("e2e_msvd-qa-oe_b2.npz")
    clips = W.synthetic_clips(2, 3, seed=int(g["seed"]))
    with torch.no_grad():
        f = v(clips.cuda())
    assert rel(f[..., :64], torch.from_numpy(g["video_features_slice"])) < 2e-2


@pytest.mark.parametrize("hw", [14, 13])
def test_block_gradient_handoff_is_bit_exact(swin, hw):
    """Consecutive blocks of a stage hand the earlier block's bf16, DropPath-scaled output gradient
    over from the later block's LN1 backward (video_swin._Handoff) instead of a separate scale-cast
    launch.  Train mode (per-clip DropPath scales, stage 3: rates > 0), whole-window and padded
    volumes: every gradient equal bit for bit to the path without the handoff where that path is
    itself run-to-run deterministic (the input gradient, the GEMM weight gradients), within 1e-6
    where it is not (LN γ/β partials and bias sums are added by atomics in arrival order)."""
    from lrce.feature_extractor import video_swin as vs
    v, _ = swin
    v.train()
    try:
        torch.manual_seed(3)
        x = torch.randn(3, 3, hw, hw, 512, device="cuda")
        R = torch.randn(3, 3, (hw + 1) // 2, (hw + 1) // 2, 1024, device="cuda")
        grads = []
        for handoff in (True, False, False):
            vs._HANDOFF = handoff
            v.zero_grad(set_to_none=True)
            torch.manual_seed(4)
            xg = x.clone().requires_grad_(True)
            (v.swin.forward_stage(2, xg, depth=4) * R).sum().backward()
            named = dict(v.named_parameters())
            grads.append([xg.grad] + [named[f"swin.layers.2.blocks.{b}.{k}"].grad.clone() for b in range(4)
                                      for k in ("mlp.fc2.weight", "mlp.fc1.bias", "norm2.weight", "attn.qkv.weight")])
        names = ["x"] + [f"{b}.{k}" for b in range(4) for k in ("fc2.w", "fc1.b", "norm2.w", "qkv.w")]
        for name, a, b, c in zip(names, *grads):
            if torch.equal(b, c):
                assert torch.equal(a, b), name
            else:
                assert rel(a, b) < 1e-6, (name, rel(a, b), rel(b, c))
    finally:
        vs._HANDOFF = True
        v.eval()
