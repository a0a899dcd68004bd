#!/usr/bin/env python
"""Fixture for the device clip assembly (csrc/video_io.hip): Pillow's resize(BILINEAR) — what the
reference's torchvision Resize((h, w)) calls on PIL images (e2e_dataset.py:60-62) — on seeded uint8
frames.  Inputs are regenerated from the seed in the test (numpy PCG64 is stable); only the PIL
outputs are stored.  Run here (Pillow 12.2.0): python tests/golden/make_video_golden.py"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))

# (name, n_frames, in_h, in_w, pick, out_h, out_w): downscale both axes (MSVD-like 240x320 -> 224),
# upscale both axes, and width unchanged (vertical pass only)
CASES = [("down", 3, 240, 320, 1, 224, 224), ("up", 2, 60, 80, 0, 112, 112), ("vonly", 2, 150, 112, 1, 112, 112)]


def frames_for(name, n, h, w):
    rng = np.random.default_rng(sum(map(ord, name)))
    base = rng.integers(0, 256, size=(n, h // 4 + 1, w // 4 + 1, 3), dtype=np.uint8)
    smooth = np.kron(base, np.ones((1, 4, 4, 1), dtype=np.uint8))[:, :h, :w]     # blocky structure
    noise = rng.integers(-12, 13, size=(n, h, w, 3))
    return np.clip(smooth.astype(np.int32) + noise, 0, 255).astype(np.uint8)


def main():
    out = {}
    for name, n, h, w, pick, oh, ow in CASES:
        fr = frames_for(name, n, h, w)
        img = Image.fromarray(fr[pick]).convert("RGB")
        out[name] = np.asarray(img.resize((ow, oh), Image.BILINEAR), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "frames_resize.npz"), **out)


if __name__ == "__main__":
    main()
