#!/usr/bin/env python
"""AdamW launch over a BERT-sized flat buffer (dev tool, GPU): microseconds per launch and effective
HBM rate (30 B per parameter: p, g, m, v read, p, m, v and the bf16 shadow written).

    python tools/adamw_bench.py [--params 110000000]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=110_000_000)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n = (a.params + 1023) // 1024 * 1024
    dev = "cuda"
    p, g = torch.randn(n, device=dev), torch.randn(n, device=dev) * 1e-3
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
    nch = n // 1024
    ct = torch.zeros(nch, dtype=torch.int32, device=dev)
    lr = torch.full((1,), 1e-4, device=dev)
    ss = torch.ones(1, device=dev)
    step = torch.ones(1, device=dev)

    def run():
        K.adamw_step(p, g, m, v, ct, lr, ss, pb, nch, 0.9, 0.999, 1e-8, 0.01, 1.0, 0.0, 0.1, 0.001, step=step)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    print(f"adamw: {n / 1e6:.0f} M params  {us:8.1f} us  "
          f"{30.0 * n / us / 1e6:6.2f} TB/s (30 B/param)", flush=True)


if __name__ == "__main__":
    main()
