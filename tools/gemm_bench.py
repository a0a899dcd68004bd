#!/usr/bin/env python
"""GEMM microbenchmark (dev tool, GPU): lrce_gemm on the step's dominant shapes vs torch.matmul
(hipBLASLt) on the same shape.  Times with HIP events over `--iters` back-to-back launches.

    python tools/gemm_bench.py [--iters 50]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import kernels as K  # noqa: E402
from lrce import _native as N  # noqa: E402

# (M, N, K, layout, flags-name): layout "fwd" = A K-major, B K-major (Y = X W^T);
# "dx" = A K-major, B N-major (dX = dY W); "dw" = A M-major, B N-major (dW = dY^T X), split-K atomic
SHAPES = [
    (4096, 4096, 4096, "fwd", ""),
    (17640, 2048, 512, "fwd", ""),
    (17640, 2048, 512, "fwd", "f32out"),
    (17640, 2048, 512, "fwd", "bias"),
    (17640, 2048, 4096, "fwd", ""),
    (17640, 2048, 512, "fwd", "bias_gelu"),
    (17640, 512, 2048, "fwd", "bias_resid"),
    (17640, 1536, 512, "fwd", "bias"),
    (17640, 512, 512, "fwd", "bias_resid"),
    (17640, 2048, 512, "dx", "dgelu"),
    (17640, 512, 512, "dx", ""),
    (17640, 512, 2048, "dx", ""),
    (17640, 512, 1536, "dx", ""),
    (512, 2048, 17640, "dw", ""),
    (2048, 512, 17640, "dw", ""),
    (1536, 512, 17640, "dw", ""),
    (282240, 512, 128, "fwd", "bias_gelu"),
    (282240, 128, 512, "fwd", "bias_resid"),
    (282240, 128, 512, "dx", "dgelu"),
    (512, 128, 282240, "dw", ""),
    (70560, 1024, 256, "fwd", "bias_gelu"),
    (4410, 4096, 1024, "fwd", "bias_gelu"),
    (320, 768, 768, "fwd", "bias"),
    (320, 3072, 768, "fwd", "bias_gelu"),
    (320, 768, 3072, "fwd", "bias"),
    (768, 768, 320, "dw", ""),
    (320, 768, 768, "dx", ""),
    (320, 768, 3072, "dx", ""),
    (320, 3072, 768, "dx", "dgelu"),
    (4500, 768, 1536, "dx", ""),
    (4500, 1536, 768, "fwd", "bias"),
    (1536, 768, 4500, "dw", ""),
    (512, 1024, 17640, "dw", ""),     # stage-2 -> 3 patch-merge reduction weight gradient
    (1024, 2048, 4410, "dw", ""),     # stage-3 -> 4 patch-merge reduction
    (768, 256, 70560, "dw", ""),      # stage-2 qkv
    (1024, 256, 70560, "dw", ""),     # stage-2 fc1
    (768, 768, 330, "dw", ""),
]


def run(M, Nn, Kk, lay, epi, iters):
    dev = "cuda"
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    if lay == "fwd":
        a = torch.rand(M, Kk, device=dev, generator=g).sub_(0.5).to(bf)
        w = torch.rand(Nn, Kk, device=dev, generator=g).sub_(0.5).to(bf)
        bias = torch.zeros(Nn, device=dev)
        resid = torch.zeros(M, Nn, device=dev) if "resid" in epi else None
        out = torch.empty(M, Nn, device=dev, dtype=torch.float32 if (resid is not None or "f32" in epi) else bf)
        pre = torch.empty(M, Nn, device=dev, dtype=bf) if "gelu" in epi else None
        f = lambda: K.linear(a, w, bias if "bias" in epi else None, out=out, gelu="gelu" in epi, pre_out=pre,  # noqa
                             resid=resid)
        ref = lambda: a @ w.t()  # noqa
    elif lay == "dx":
        dy = torch.rand(M, Kk, device=dev, generator=g).sub_(0.5).to(bf)    # [M, N_out]
        w = torch.rand(Kk, Nn, device=dev, generator=g).sub_(0.5).to(bf)    # [N_out, K_in]
        pre = torch.rand(M, Nn, device=dev, generator=g).to(bf) if "dgelu" in epi else None
        out = torch.empty(M, Nn, device=dev, dtype=bf)
        f = lambda: K.linear_dx(dy, w, out=out, dgelu_pre=pre)  # noqa
        ref = lambda: dy @ w  # noqa
    else:  # dw: dW[M=out, N=in] += dY[K=tokens, M]^T X[K, N]
        dy = torch.rand(Kk, M, device=dev, generator=g).sub_(0.5).to(bf)
        x = torch.rand(Kk, Nn, device=dev, generator=g).sub_(0.5).to(bf)
        dw = torch.zeros(M, Nn, device=dev)
        f = lambda: K.linear_dw(dy, x, dw)  # noqa
        ref = lambda: dy.t() @ x  # noqa
    res = []
    for fn in (f, ref):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        res.append(ms)
    fl = 2.0 * M * Nn * Kk
    print(f"{M:7d} {Nn:6d} {Kk:7d} {lay:3s} {epi:10s}  lrce {res[0]*1e3:8.1f} us {fl/res[0]/1e9:7.1f} TF/s   "
          f"torch {res[1]*1e3:8.1f} us {fl/res[1]/1e9:7.1f} TF/s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--only", type=int, default=-1)
    ap.add_argument("--first", type=int, default=1000)
    a = ap.parse_args()
    N.lib()
    for i, s in enumerate(SHAPES):
        if (a.only < 0 or a.only == i) and i < a.first:
            run(*s, a.iters)


if __name__ == "__main__" and not os.environ.get("DW_SWEEP"):
    main()


def dw_split_sweep(iters=20):
    """dW = dY^T X at the Swin stage-3 shapes: split-K factor vs time (atomic f32 accumulation)."""
    dev = "cuda"
    for (M, Nn, Kk) in [(512, 2048, 17640), (2048, 512, 17640), (512, 512, 17640), (1536, 512, 17640),
                        (512, 128, 282240), (256, 1024, 70560)]:
        dy = torch.rand(Kk, M, device=dev).sub_(0.5).to(torch.bfloat16)
        x = torch.rand(Kk, Nn, device=dev).sub_(0.5).to(torch.bfloat16)
        dw = torch.zeros(M, Nn, device=dev)
        line = f"dw {M:5d} {Nn:5d} {Kk:6d}: auto {K._split_for(M, Nn, Kk)}"
        ws = torch.empty(128 * M * Nn, device=dev) if os.environ.get("DW_SLAB") else None
        for split in (1, 2, 4, 8, 16, 32, 64, 128):
            fl = N.EPI_ATOMIC if split > 1 else N.EPI_ACCUM
            f = lambda: K.gemm(dy, x, dw, M, Nn, Kk, a_kmajor=False, b_kmajor=False, lda=M, ldb=Nn, ldc=Nn,  # noqa
                               flags=fl, split_k=split, workspace=ws)
            for _ in range(2):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / iters
            line += f"  s{split}:{ms * 1e3:6.1f}us"
        print(line, flush=True)


if __name__ == "__main__" and os.environ.get("DW_SWEEP"):
    dw_split_sweep()
