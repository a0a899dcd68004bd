#!/usr/bin/env python
"""Patch im2col microbenchmark (dev tool, GPU): lrce_patch_im2col at the bs-10 step's shape (30 clips of
5 frames, 224^2, normalised), HIP-event timed; bytes = the f32 clips read + the bf16 patches written."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import kernels as K  # noqa: E402


def main():
    dev = "cuda"
    B, S, T, H, W = 10, 3, 5, 224, 224
    clips = torch.rand(B, S, T, 3, H, W, device=dev)
    ntok = B * S * ((T + 1) // 2) * (H // 4) * (W // 4)
    patches = torch.empty(ntok, 96, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        K.patch_im2col(clips, patches)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 50
    e0.record()
    for _ in range(it):
        K.patch_im2col(clips, patches)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    gb = (clips.numel() * 4 + patches.numel() * 2) / 1e9
    print(f"patch_im2col {ntok} tokens: {ms * 1e3:.1f} us  {gb / ms:.2f} TB/s")


if __name__ == "__main__":
    main()
