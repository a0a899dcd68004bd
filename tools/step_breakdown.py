#!/usr/bin/env python
"""Per-launch-shape GEMM breakdown of one eager bench step (dev tool, GPU).

    python tools/step_breakdown.py [--batch-size 10] [--top 60]

Prints, for every distinct (M, N, K, batch, A/B layout, A dtype, split-K, epilogue flags) GEMM
launch of the training step: calls, total ms per step, achieved TFLOP/s."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from lrce import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=10)
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model, opt, reducer, batch = bench.build(a.batch_size, dev, torch.bfloat16)
    for _ in range(2):
        bench.train_step(model, opt, reducer, batch)
    torch.cuda.synchronize()
    kt = K.KernelTimer("gemm", "gemm_f32", "wattn_fwd", "wattn_qkv_fwd", "wattn_bwd", detail=True)
    with kt:
        bench.train_step(model, opt, reducer, batch)
    rows = kt.breakdown()
    tot = sum(r[3] for r in rows)
    print(f"total timed {tot:.2f} ms/step over {sum(r[2] for r in rows)} launches")
    print(f"{'kernel':10s} {'M':>7s} {'N':>6s} {'K':>7s} {'bt':>3s} lay      sk flags calls   ms   TF/s")
    for name, key, n, t, tf in rows[:a.top]:
        if key is None or len(key) != 9:
            print(f"{name:10s} {str(key or ''):48s} {n:5d} {t:6.3f} {tf:7.1f}")
            continue
        m, nn, k, b, la, lb, ad, sk, fl = key
        print(f"{name:10s} {m:7d} {nn:6d} {k:7d} {b:3d} {la}{lb}{ad} {sk:3d} {fl:5d} {n:5d} {t:6.3f} {tf:7.1f}")


if __name__ == "__main__":
    main()
