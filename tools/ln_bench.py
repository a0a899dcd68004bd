#!/usr/bin/env python
"""LayerNorm-backward microbenchmark (dev tool, GPU): the Swin block's norm2 backward shape
(dy, x f32, + residual gradient, + bf16 copy of dx) per stage, with and without the dw/db
reductions, against the algorithmic HBM bytes.

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

SHAPES = [(282240, 128), (70560, 256), (17640, 512), (4410, 1024), (12000, 768), (320, 768)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = "cuda"
    for R, C in SHAPES:
        x = torch.randn(R, C, device=dev)
        dy = torch.randn(R, C, device=dev)
        dres = torch.randn(R, C, device=dev)
        w = torch.rand(C, device=dev) + 0.5
        b = torch.zeros(C, device=dev)
        _, mean, rstd = K.layernorm(x, w, b, 1e-5, out_f32=True)
        dx = torch.empty_like(x)
        dx16 = torch.empty(R, C, dtype=torch.bfloat16, device=dev)
        dw = torch.zeros(C, device=dev)
        db = torch.zeros(C, device=dev)
        line = f"ln_bwd {R:7d} x {C:5d}:"
        for name, kw, nbytes in (
                ("plain", {}, 3 * 4),
                ("dwdb", dict(dw=dw, db=db), 3 * 4),
                ("dres+dx16+dwdb", dict(dres=dres, dx16=dx16, dw=dw, db=db), 4 * 4 + 2)):
            ms = timeit(lambda: K.layernorm_bwd(dy, x, mean, rstd, w, dx, **kw), a.iters)
            gbs = R * C * nbytes / ms / 1e6
            line += f"  {name} {ms * 1e3:7.1f} us {gbs:6.0f} GB/s"
        print(line, flush=True)
        ms = timeit(lambda: K.layernorm(x, w, b, 1e-5, out=dx), a.iters)
        print(f"ln_fwd {R:7d} x {C:5d}: {ms * 1e3:7.1f} us {R * C * 8 / ms / 1e6:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
