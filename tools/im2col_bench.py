#!/usr/bin/env python
"""Elementwise microbenchmarks (dev tool, GPU), HIP-event timed: lrce_patch_im2col at the bs-10 step's
shape (30 clips of 5 frames, 224^2, normalised; bytes = the f32 clips read + the bf16 patches written)
and lrce_scale_cast_bf16 at the Swin stage shapes with per-clip row scales (the DropPath-scaled bf16
copy of a block's output gradient)."""
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
    for rows, cols in ((282240, 128), (70560, 256), (15680, 512), (3920, 1024)):
        x = torch.randn(rows, cols, device=dev)
        sc = torch.rand(30, device=dev)
        y = torch.empty(rows, cols, device=dev, dtype=torch.bfloat16)
        f = lambda: K.scale_cast_bf16(x, sc, rows // 30, out=y)   # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(it):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        print(f"scale_cast_bf16 {rows}x{cols}: {ms * 1e3:.1f} us  {rows * cols * 6 / 1e9 / ms:.2f} TB/s")


if __name__ == "__main__":
    main()
