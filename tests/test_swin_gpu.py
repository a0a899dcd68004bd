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
