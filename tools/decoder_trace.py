#!/usr/bin/env python
"""Phase timeline of the fused decoder block kernels (dev tool, GPU): runs the LRCE OE fusion head
(bench shapes: 10 rows, temporal scale 3, 32 question tokens, dropout on) forward + backward, with
lrce_dec_set_trace on for one step, and prints per kernel and per mark the median / max over
workgroups of (mark time - the launch's first start), in us (s_memrealtime: 10 ns resolution).

    python tools/decoder_trace.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import _native as N  # noqa: E402
from lrce.models.fusionv3 import LRCEOpenEnded  # noqa: E402

MARKS = {
    "sa_fwd": ["start", "x0 ready", "v proj", "slice landed", "out partial", "published", "last done"],
    "ca_fwd": ["start", "x1 ready", "q proj", "softmax", "V/slice landed", "ctx", "out partial", "published", "last done",
               "(row loaded)", "(bulk issued)"],
    "ca_bwd": ["start", "LN2 bwd", "K/V/slice landed", "dctx", "P/dS", "dq, dK/dV", "dx1 partial", "published", "last done",
               "(rows loaded)", "(bulk issued)", "(LN reduced)"],
    "sa_bwd": ["start", "LN1 bwd", "slice landed", "dx0 partial", "published", "last done"],
}


def main():
    B, L = 10, 32
    torch.manual_seed(0)
    m = LRCEOpenEnded(768, 1000, 0.1, (7, 7), 1024, 5, [3], L).cuda().train()
    vf = torch.randn(B, 3, 3, 49, 1024, device="cuda")
    tf = torch.randn(B, L, 768, device="cuda")

    def step():
        m.zero_grad(set_to_none=True)
        y = m(vf, tf, None)
        y.float().sum().backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    buf = torch.zeros(4 * 1024 * 16, dtype=torch.int64, device="cuda")
    N.call("lrce_dec_set_trace", buf.data_ptr())
    step()
    torch.cuda.synchronize()
    N.call("lrce_dec_set_trace", None)
    tr = buf.view(4, 1024, 16).cpu()
    nwg = B * 12
    for k, (name, marks) in enumerate(MARKS.items()):
        t = tr[k, :nwg, :len(marks)].double()
        t0 = t[:, 0].min()
        print(f"{name}: start skew (max - min over {nwg} workgroups) {(t[:, 0].max() - t0).item() / 100:.2f} us")
        for i, mk in enumerate(marks):
            col = t[:, i]
            ok = col > 0
            if not ok.any():
                continue
            d = (col[ok] - t0) / 100.0
            print(f"   {i} {mk:18s} median {d.median().item():7.2f}  max {d.max().item():7.2f} us  ({int(ok.sum())} wg)")


if __name__ == "__main__":
    main()
