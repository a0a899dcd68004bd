"""Device clip assembly (csrc/video_io.hip, lrce/dataset/video.py) vs Pillow and the reference's
frame selection (e2e_dataset.py:60-111): bit-exact uint8 resample, exact [0, 1] floats, and the
(S, fpc, 3, 224, 224) clip layout the video extractor consumes."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]
sys.path.insert(0, GOLDEN)


def test_frames_resize_matches_pillow_bit_exact():
    from make_video_golden import CASES, frames_for
    from lrce import kernels as K
    g = np.load(os.path.join(GOLDEN, "frames_resize.npz"))
    for name, n, h, w, pick, oh, ow in CASES:
        fr = torch.from_numpy(frames_for(name, n, h, w)).cuda()
        out = K.frames_resize(fr, torch.tensor([pick], dtype=torch.int32, device="cuda"), oh, ow)
        ref = torch.from_numpy(g[name]).permute(2, 0, 1).float().div(255.0)   # ToTensor
        assert torch.equal(out[0].cpu(), ref), name


def test_clips_from_frames_layout_and_selection():
    from oracle.video_resize import multiscale_frame_indices, pil_bilinear_resize
    from lrce.dataset.video import clips_from_frames
    rng = np.random.default_rng(7)
    T, H, W = 37, 96, 128
    fr = rng.integers(0, 256, size=(T, H, W, 3), dtype=np.uint8)
    clips = clips_from_frames(torch.from_numpy(fr).cuda(), 5, [1, 2, 3], (64, 80))
    assert clips.shape == (6, 5, 3, 64, 80) and clips.dtype == torch.float32
    idx = multiscale_frame_indices(T, 5, [1, 2, 3])
    got = clips.view(30, 3, 64, 80).cpu()
    for f in (0, 7, 18, 29):
        ref = torch.from_numpy(pil_bilinear_resize(fr[idx[f]], 64, 80)).permute(2, 0, 1).float().div(255.0)
        assert torch.equal(got[f], ref), f


def test_frames_resize_rejects_bad_input():
    from lrce import kernels as K
    from lrce import _native as N
    fr = torch.zeros(2, 4000, 4000, 3, dtype=torch.uint8, device="cuda")
    with pytest.raises(N.NativeError):
        K.frames_resize(fr, torch.zeros(1, dtype=torch.int32, device="cuda"), 224, 224)   # 17.9x downscale
    with pytest.raises(N.NativeError):
        K.frames_resize(fr.cpu(), torch.zeros(1, dtype=torch.int32), 224, 224)            # no CPU fallback
