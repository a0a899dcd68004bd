#!/usr/bin/env python
"""Phase timeline of the window-attention backward (WATTN_FWD=1: the fused qkv + attention forward)
(dev tool, GPU): one lrce_wattn_bwd launch at a
Swin-B stage shape of the bs=10 step with lrce_wattn_set_trace on; prints the launch span, the
number of workgroups resident at once, and per mark the median / p90 time since the workgroup's own
start (s_memrealtime, 100 MHz: 10 ns resolution).

    make -C vqa-lrce-kbs-2023_amd/csrc BUILD=build_trace EXTRA=-DLRCE_WATTN_TRACE OUT=../../tools/_trace.so
    LRCE_NATIVE_LIB=$PWD/tools/_trace.so WATTN_STAGE=2 python tools/wattn_trace.py   # 0..3: (1920, 4) .. (30, 32)
(the marks are compiled in only with -DLRCE_WATTN_TRACE: they cost registers the product kernel keeps)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import _native as N  # noqa: E402
from lrce import kernels as K  # noqa: E402
from lrce.feature_extractor.video_swin import relative_position_index  # noqa: E402

STAGES = [(1920, 4), (480, 8), (120, 16), (30, 32)]
MARKS = ["start", "prologue", "step 0", "step 1", "step 2", "step 3", "step 4", "stores", "bins out"]
FWD_MARKS = ["start", "GEMM", "epilogue", "qkv stored", "attention", "O stored"]   # WATTN_FWD=1: the fused forward


def main():
    dev = "cuda"
    n, hd = 147, 32
    n_win, nH = STAGES[int(os.environ.get("WATTN_STAGE", "2"))]
    C = nH * hd
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = (torch.randn(n_win * n, 3 * C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    n_pat = 4
    table = torch.randn(2535, nH, device=dev, generator=g) * 0.02
    idx = relative_position_index((8, 7, 7)).to(dev)
    region = torch.randint(0, 3, (n_pat, n), device=dev, generator=g, dtype=torch.int32)
    win_pat = torch.randint(0, n_pat, (n_win,), device=dev, generator=g, dtype=torch.int32)
    be = K.wattn_bias_elems(n_pat, nH)
    bf_ = torch.empty(be, device=dev)
    bbh = torch.empty(be, device=dev, dtype=torch.float16)
    K.wattn_bias_build(table, idx, n, nH, region, n_pat, bf_, bbh)
    out = torch.empty(n_win * n, C, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(n_win * nH * 160, device=dev)
    K.wattn_fwd_grouped(qkv, bf_, K.wattn_groups(win_pat, n_win, dev), out, lse, n_win, n, nH)
    dout = (torch.randn(n_win * n, C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    win = (3, 7, 7)
    dbp = torch.empty(K.wattn_dbias_part_elems(n_win, nH, win), device=dev)

    marks = MARKS
    if os.environ.get("WATTN_FWD"):
        marks = FWD_MARKS
        x = (torch.randn(n_win * n, C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        wq = (torch.randn(3 * C, C, device=dev, generator=g) / C ** 0.5).to(torch.bfloat16)
        bq = torch.zeros(3 * C, device=dev)
        bfh = torch.empty(be, device=dev, dtype=torch.float16)
        K.wattn_bias_build(table, idx, n, nH, region, n_pat, torch.empty(be, device=dev), bfh)
        order = torch.argsort(win_pat.long(), stable=True).int()

        def run():
            K.wattn_qkv_fwd(x, wq, bq, 0.25, bfh, win_pat, qkv, out, lse, n_win, n, nH, win_order=order)
    else:
        def run():
            K.wattn_bwd(qkv, out, dout, lse, bbh, win_pat, dqkv, dbp, n_win, n, nH, win)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    nwg = n_win * nH // (1 if nH % 2 else 2)   # two heads per workgroup when nH is even (both kernels)
    buf = torch.zeros(nwg * 16, dtype=torch.int64, device=dev)
    N.call("lrce_wattn_set_trace", buf.data_ptr())
    run()
    torch.cuda.synchronize()
    N.call("lrce_wattn_set_trace", None)
    last = len(marks) - 1
    tr = buf.view(nwg, 16)[:, :len(marks)].double().cpu() / 100.0   # us
    t0 = tr[:, 0]
    span = (tr[:, last].max() - t0.min()).item()
    print(f"windows {n_win} heads {nH}: {nwg} workgroups, launch span {span:.1f} us")
    # residency: workgroups alive at each workgroup's start
    st, en = t0.sort().values, tr[:, last].sort().values
    alive = torch.arange(1, nwg + 1, dtype=torch.float64) - torch.searchsorted(en, st, right=True).double()
    print(f"resident workgroups at a start: median {alive.median().item():.0f}  max {alive.max().item():.0f}")
    life = tr[:, last] - t0
    print(f"workgroup lifetime: median {life.median().item():.2f}  p90 {life.quantile(0.9).item():.2f} us")
    hw = buf.view(nwg, 16)[:, 10].cpu()
    xcc = buf.view(nwg, 16)[:, 11].cpu() & 0xF
    cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | (xcc << 8)
    ncu = len(torch.unique(cu))
    best = 0
    for c in torch.unique(cu)[:32].tolist():   # max overlap of workgroup lifetimes on one CU
        m = cu == c
        ev = sorted([(a, 1) for a in t0[m].tolist()] + [(b, -1) for b in tr[m, last].tolist()], key=lambda e: (e[0], e[1]))
        cur = 0
        for _, d in ev:
            cur += d
            best = max(best, cur)
    print(f"distinct CUs used {ncu}; max workgroups alive on one CU (first 32 CUs) {best}")
    prev = None
    for i, mk in enumerate(marks):
        d = tr[:, i] - t0
        step = "" if prev is None else f"   (+{(d - prev).median().item():.2f} median)"
        print(f"  {i} {mk:10s} median {d.median().item():7.2f}  p90 {d.quantile(0.9).item():7.2f} us{step}")
        prev = d


if __name__ == "__main__":
    main()
