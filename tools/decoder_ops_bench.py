#!/usr/bin/env python
"""Decoder query-path op microbenchmark (dev tool, GPU): each op replayed 50x from a captured HIP
graph (the bench's launch mode), so the per-launch time includes the in-graph launch gap."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import kernels as K  # noqa: E402


def graph_time(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


def main():
    dev = "cuda"
    B, E, FF = 10, 768, 3072
    x = torch.randn(B, E, device=dev)
    w = torch.randn(E, E, device=dev) * 0.02
    w1 = torch.randn(FF, E, device=dev) * 0.02
    w2 = torch.randn(E, FF, device=dev) * 0.02
    b = torch.zeros(E, device=dev)
    b1 = torch.zeros(FF, device=dev)
    y = torch.empty(B, E, device=dev)
    g = torch.empty(B, FF, device=dev)
    pre = torch.empty(B, FF, dtype=torch.bfloat16, device=dev)
    gw = torch.zeros(E, E, device=dev)
    gw1 = torch.zeros(FF, E, device=dev)
    res = []
    res.append(("skinny fwd 10x768x768", graph_time(lambda: K.linear(x, w, b, out=y, out_f32=True))))
    res.append(("skinny fwd 10x3072x768 gelu", graph_time(lambda: K.linear(x, w1, b1, out=g, gelu=True, pre_out=pre, out_f32=True))))
    res.append(("skinny fwd 10x768x3072", graph_time(lambda: K.linear(g, w2, b, out=y, out_f32=True))))
    res.append(("skinny dX 10x768x768", graph_time(lambda: K.linear_dx(y, w, out=x))))
    res.append(("skinny dX 10x768x3072", graph_time(lambda: K.linear_dx(g, w2.t().contiguous() if False else w1, out=x))))
    res.append(("outer dW 768x768 K=10", graph_time(lambda: K.linear_dw(y, x, gw, bias_grad=b))))
    res.append(("outer dW 3072x768 K=10", graph_time(lambda: K.linear_dw(g, x, gw1, bias_grad=b1))))
    x30 = torch.randn(30, E, device=dev)
    y30 = torch.randn(30, E, device=dev)
    res.append(("outer dW 768x768 K=30", graph_time(lambda: K.linear_dw(y30, x30, gw, bias_grad=b))))
    res.append(("dropout 10x768", graph_time(lambda: K.dropout(y, 0.1, 5, out=y))))
    ln_w, ln_b = torch.ones(E, device=dev), torch.zeros(E, device=dev)
    res.append(("layernorm 10x768", graph_time(lambda: K.layernorm(y, ln_w, ln_b, 1e-12, out_f32=True))))
    # rotating weights (36 distinct copies, as the 12 layers x 3 steps of one decoder pass): cold in L2
    nrot = 36
    ws32 = [torch.randn(E, E, device=dev) * 0.02 for _ in range(nrot)]
    ws16 = [t.half() for t in ws32]
    w1s16 = [(torch.randn(FF, E, device=dev) * 0.02).half() for _ in range(nrot)]
    ctr = [0]

    def rot(ws, fn):
        def f():
            ctr[0] = (ctr[0] + 1) % nrot
            fn(ws[ctr[0]])
        return f
    res.append(("rot skinny fwd 768x768 f32 W", graph_time(rot(ws32, lambda wt: K.linear(x, wt, b, out=y, out_f32=True)), reps=36)))
    res.append(("rot skinny fwd 768x768 fp16 W", graph_time(rot(ws16, lambda wt: K.linear(x, wt, b, out=y, out_f32=True)), reps=36)))
    res.append(("L2 skinny fwd 768x768 fp16 W", graph_time(lambda: K.linear(x, ws16[0], b, out=y, out_f32=True))))
    res.append(("rot skinny fwd 3072x768 fp16 W gelu", graph_time(rot(w1s16, lambda wt: K.linear(x, wt, b1, out=g, gelu=True, pre_out=pre, out_f32=True)), reps=36)))
    pro_m, pro_r = torch.empty(B, device=dev), torch.empty(B, device=dev)
    yo = torch.empty(B, E, device=dev)
    res.append(("rot skinny_ln fwd 768x768 fp16 W", graph_time(rot(ws16, lambda wt: K.linear(
        x, wt, b, out=y, out_f32=True, ln=K.ln_fwd_prologue(ln_w, ln_b, 1e-12, mean=pro_m, rstd=pro_r, y_out=yo))), reps=36)))
    res.append(("empty-ish: dropout p=0 10x768", graph_time(lambda: K.dropout(y, 0.0, 5, out=y))))
    for name, us in res:
        print(f"{name:32s} {us:7.2f} us/launch", flush=True)


if __name__ == "__main__":
    main()
