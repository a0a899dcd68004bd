#!/usr/bin/env python
"""Recurrent-decoder microbenchmark (dev tool, GPU): the LRCE fusion head of the msvd-qa-oe bench
workload (bs 10, 3 clips, 33 question keys, dropout 0.5, train mode) forward + backward, per decoder
implementation (LRCE_DEC_FUSED = step | blocks | 0): wall time per head step (eager) and, through
KernelTimer("decoder"), the mean duration of the decoder launches (the persistent step kernels, or
the per-block kernels), split into forward / backward.

    python tools/decoder_step_bench.py [--modes step,blocks] [--iters 10] [--batch 10]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import kernels as K  # noqa: E402


def run(mode, iters, B, task):
    from lrce.models.fusionv3 import LRCEOpenEnded, LRCEMultipleChoice
    os.environ["LRCE_DEC_FUSED"] = mode
    torch.manual_seed(0)
    if task == "mc":
        m = LRCEMultipleChoice(768, 1, 0.5, (7, 7), 1024, 5, [3], 40).cuda().train()
        tf = torch.randn(B, 5, 40, 768, device="cuda")
    else:
        m = LRCEOpenEnded(768, 1000, 0.5, (7, 7), 1024, 5, [3], 32).cuda().train()
        tf = torch.randn(B, 32, 768, device="cuda")
    vf = torch.randn(B, 3, 3, 49, 1024, device="cuda")

    def step():
        vg, tg = vf.detach().requires_grad_(True), tf.detach().requires_grad_(True)
        y = m(vg, tg, None)
        y.float().sum().backward()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    code = K.dec_step_status("cuda")
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters * 1e3
    kt = K.KernelTimer("decoder")
    with kt:
        step()
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in kt.events["decoder"]]
    code = code or K.dec_step_status("cuda")
    return wall, ms, code


FWD_MARKS = ["A0", "A-ffn-wait", "A-row-wait", "A-end", "B-row-wait", "B-end", "C-wait", "C-end"]
BWD_MARKS = ["FB0", "FB-wait", "FB-end", "CB-sl-wait", "CB-row-wait", "CB-end", "SB-row-wait", "SB-end"]


def trace(B, task):
    from lrce import _native as N
    import numpy as np
    buf = torch.zeros(2 * 128 * 16 * 8, dtype=torch.int64, device="cuda")
    N.call("lrce_dec_step_set_trace", N.ptr(buf))
    try:
        run("step", 1, B, task)
    finally:
        N.call("lrce_dec_step_set_trace", None)
    torch.cuda.synchronize()
    t = buf.view(2, 128, 16, 8).cpu().numpy().astype(np.float64)
    G = N.lib().lrce_dec_step_grid(B)
    for d, names in ((0, FWD_MARKS), (1, BWD_MARKS)):
        x = t[d, :G]
        valid = x[x > 0]
        t0 = valid.min()
        print(f"== {'forward' if d == 0 else 'backward'} (last launch), us from launch start: median / max over workgroups")
        layers = list(range(13) if d == 0 else range(12, -1, -1)) + [14]
        prev_end = None
        for l in layers:
            row = []
            for i, nm in enumerate(names if l != 14 else [f"s{k}" for k in range(8)]):
                v = x[:, l, i]
                v = v[v > 0]
                if len(v):
                    row.append(f"{nm} {(np.median(v) - t0) / 100:7.1f}/{(v.max() - t0) / 100:7.1f}")
            if row:
                print(f"L{l:2d}  " + "  ".join(row) if l != 14 else "FFN sub-phases of layer 1 (marks 0-7): " + "  ".join(row))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="step,blocks")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=10)
    ap.add_argument("--task", default="oe")
    ap.add_argument("--trace", action="store_true", help="phase timestamps of the last forward / backward step launch")
    a = ap.parse_args()
    if a.trace:
        trace(a.batch, a.task)
        return
    for mode in a.modes.split(","):
        wall, ms, code = run(mode, a.iters, a.batch, a.task)
        n = len(ms)
        half = n // 2
        print(f"{mode:7s} head fwd+bwd {wall:7.3f} ms (eager)  decoder launches {n}: total {sum(ms):.3f} ms  "
              f"fwd {sum(ms[:half]):.3f}  bwd {sum(ms[half:]):.3f}  status {code:#x}", flush=True)
        if mode == "step":
            print("   per launch (ms):", " ".join(f"{x:.3f}" for x in ms), flush=True)


if __name__ == "__main__":
    main()
