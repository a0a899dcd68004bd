#!/usr/bin/env python
"""Phase timeline of one LDS-DMA GEMM launch (dev tool, GPU): a gemm_bench.py shape with
lrce_gemm_set_trace on; prints the launch span, workgroups resident at once, and per mark the
median / p90 time since the workgroup's own start (s_memrealtime, 100 MHz).

    make -C vqa-lrce-kbs-2023_amd/csrc BUILD=build_trace EXTRA="-DLRCE_WATTN_TRACE -DLRCE_GEMM_TRACE" OUT=../../tools/_trace.so
    LRCE_NATIVE_LIB=$PWD/tools/_trace.so python tools/gemm_trace.py 5 9 16      (gemm_bench.py SHAPES indices)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import _native as N  # noqa: E402
from lrce import kernels as K  # noqa: E402
import gemm_bench as GB  # noqa: E402

MARKS = ["start", "tile 0 in", "K loop", "issued", "drained"]


def trace(idx):
    M, Nn, Kk, lay, epi = GB.SHAPES[idx]
    dev = "cuda"
    bf = torch.bfloat16
    if lay == "fwd":
        a = torch.rand(M, Kk, device=dev).sub_(0.5).to(bf)
        w = torch.rand(Nn, Kk, device=dev).sub_(0.5).to(bf)
        bias = torch.zeros(Nn, device=dev)
        resid = torch.zeros(M, Nn, device=dev) if "resid" in epi else None
        out = torch.empty(M, Nn, device=dev, dtype=torch.float32 if (resid is not None or "f32" in epi) else bf)
        pre = torch.empty(M, Nn, device=dev, dtype=bf) if "gelu" in epi else None
        f = lambda: K.linear(a, w, bias if "bias" in epi else None, out=out, gelu="gelu" in epi, pre_out=pre, resid=resid)  # noqa
    elif lay == "dx":
        dy = torch.rand(M, Kk, device=dev).sub_(0.5).to(bf)
        w = torch.rand(Kk, Nn, device=dev).sub_(0.5).to(bf)
        pre = torch.rand(M, Nn, device=dev).to(bf) if "dgelu" in epi else None
        out = torch.empty(M, Nn, device=dev, dtype=bf)
        f = lambda: K.linear_dx(dy, w, out=out, dgelu_pre=pre)  # noqa
    else:
        dy = torch.rand(Kk, M, device=dev).sub_(0.5).to(bf)
        x = torch.rand(Kk, Nn, device=dev).sub_(0.5).to(bf)
        dw = torch.zeros(M, Nn, device=dev)
        f = lambda: K.linear_dw(dy, x, dw)  # noqa
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    nmax = 65536
    buf = torch.zeros(nmax * 8, dtype=torch.int64, device=dev)
    N.call("lrce_gemm_set_trace", buf.data_ptr())
    f()
    torch.cuda.synchronize()
    N.call("lrce_gemm_set_trace", None)
    tr = buf.view(nmax, 8)
    nwg = int((tr[:, 0] != 0).sum().item())
    tr = tr[:nwg]
    t = tr[:, :5].double().cpu() / 100.0
    t0 = t[:, 0]
    span = (t[:, 4].max() - t0.min()).item()
    print(f"== {M}x{Nn}x{Kk} {lay} {epi}: {nwg} workgroups, launch span {span:.1f} us")
    st, en = t0.sort().values, t[:, 4].sort().values
    alive = torch.arange(1, nwg + 1, dtype=torch.float64) - torch.searchsorted(en, st, right=True).double()
    print(f"resident workgroups at a start: median {alive.median().item():.0f}  max {alive.max().item():.0f}")
    life = t[:, 4] - t0
    print(f"workgroup lifetime: median {life.median().item():.2f}  p90 {life.quantile(0.9).item():.2f} us")
    rel_start = t0 - t0.min()
    print(f"workgroup starts: p10 {rel_start.quantile(0.1).item():.1f}  median {rel_start.median().item():.1f}  "
          f"p90 {rel_start.quantile(0.9).item():.1f} us after the first")
    prev = None
    for i, mk in enumerate(MARKS):
        d = t[:, i] - t0
        stp = "" if prev is None else f"   (+{(d - prev).median().item():.2f} median)"
        print(f"  {i} {mk:10s} median {d.median().item():7.2f}  p90 {d.quantile(0.9).item():7.2f} us{stp}")
        prev = d


def main():
    for a in sys.argv[1:] or ["5", "9", "16", "6"]:
        trace(int(a))


if __name__ == "__main__":
    main()
