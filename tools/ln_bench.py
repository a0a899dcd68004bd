#!/usr/bin/env python
"""LayerNorm microbenchmark (dev tool, GPU): lrce LayerNorm backward / forward at the Swin-B step's
row x column shapes, isolated (HIP events over back-to-back launches), against torch's native
layer_norm backward on the same shape.  Bytes are the algorithmic ones of the lrce call.

    python tools/ln_bench.py [--iters 30]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import kernels as K  # noqa: E402

SHAPES = [(250880, 128), (62720, 256), (15680, 512), (3920, 1024), (62720, 512), (15680, 1024), (3920, 2048), (320, 768)]


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = "cuda"
    for R, C in SHAPES:
        x = torch.randn(R, C, device=dev)
        w = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev)
        y, mean, rstd = K.layernorm(x, w, b, 1e-5, out_f32=True)
        dres = torch.randn(R, C, device=dev)
        dx = torch.empty(R, C, device=dev)
        dx16 = torch.empty(R, C, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(C, device=dev)
        db = torch.zeros(C, device=dev)
        for dyt in (torch.float32, torch.bfloat16):
            dy = torch.randn(R, C, device=dev).to(dyt)
            f = lambda: K.layernorm_bwd(dy, x, mean, rstd, w, dx, dres=dres, dw=dw, db=db, dx16=dx16)  # noqa
            us = timed(f, a.iters)
            by = R * C * (4 + dy.element_size() + 4 + 4 + 2) + 8 * R
            print(f"ln_bwd {R:7d} x {C:5d} dy {str(dyt)[6:]:9s} {us:8.1f} us {by / us / 1e3:7.0f} GB/s", flush=True)
        xt = x.clone()
        dyt = torch.randn(R, C, device=dev)
        tf = lambda: torch.ops.aten.native_layer_norm_backward(dyt, xt, [C], mean.view(R, 1), rstd.view(R, 1), w, b,  # noqa
                                                               [True, True, True])
        us = timed(tf, a.iters)
        by = R * C * (4 + 4 + 4) + 8 * R
        print(f"torch  {R:7d} x {C:5d} dy f32       {us:8.1f} us {by / us / 1e3:7.0f} GB/s (x, dy read; dx write)", flush=True)
        y16 = torch.empty(R, C, device=dev, dtype=torch.bfloat16)
        f = lambda: K.layernorm(x, w, b, 1e-5, out=y16)  # noqa
        us = timed(f, a.iters)
        by = R * C * (4 + 2) + 8 * R
        print(f"ln_fwd {R:7d} x {C:5d} y bf16    {us:8.1f} us {by / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
