#!/usr/bin/env python
"""Window-attention kernel microbenchmark (dev tool, GPU): lrce_wattn_fwd / _bwd at the four Swin-B
stage shapes of the bs=10 msvd step (n = 147 tokens, d = 32), HIP-event timed; algorithmic TFLOP/s =
4 n^2 d (fwd) / 8 n^2 d (bwd) per (window, head) as in bench.py."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce import kernels as K  # noqa: E402
from lrce.feature_extractor.video_swin import relative_position_index  # noqa: E402

STAGES = [(1920, 4), (480, 8), (120, 16), (30, 32)]   # (windows, heads) at bs=10 x 3 clips


def timeit(f, iters=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    dev = "cuda"
    n, hd = 147, 32
    tot_f = tot_b = fl_f = fl_b = 0.0
    only = os.environ.get("WATTN_STAGE")
    stages = [STAGES[int(only)]] if only else STAGES
    for n_win, nH in stages:
        C = nH * hd
        g = torch.Generator(device=dev).manual_seed(0)
        qkv = (torch.randn(n_win * n, 3 * C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        n_pat = 4
        table = torch.randn(2535, nH, device=dev, generator=g) * 0.02
        idx = relative_position_index((8, 7, 7)).to(dev)
        region = torch.randint(0, 3, (n_pat, n), device=dev, generator=g, dtype=torch.int32)
        win_pat = torch.randint(0, n_pat, (n_win,), device=dev, generator=g, dtype=torch.int32)
        be = K.wattn_bias_elems(n_pat, nH)
        bf_, bb_ = torch.empty(be, device=dev), torch.empty(be, device=dev)
        K.wattn_bias_build(table, idx, n, nH, region, n_pat, bf_, bb_)
        bfh = torch.empty(be, device=dev, dtype=torch.float16)
        bbh = torch.empty(be, device=dev, dtype=torch.float16)
        K.wattn_bias_build(table, idx, n, nH, region, n_pat, bfh, bbh)   # the product's fp16 tiles
        order = torch.argsort(win_pat.long(), stable=True).int()
        out = torch.empty(n_win * n, C, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(n_win * nH * 160, device=dev)
        dout = (torch.randn(n_win * n, C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        dqkv = torch.empty_like(qkv)
        win = (3, 7, 7)
        dbp = torch.empty(K.wattn_dbias_part_elems(n_win, nH, win), device=dev)
        groups = K.wattn_groups(win_pat, n_win, dev)
        tf = timeit(lambda: K.wattn_fwd_grouped(qkv, bf_, groups, out, lse, n_win, n, nH))
        x = (torch.randn(n_win * n, C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        wq = (torch.randn(3 * C, C, device=dev, generator=g) / C ** 0.5).to(torch.bfloat16)
        bq = torch.zeros(3 * C, device=dev)
        tq = timeit(lambda: K.wattn_qkv_fwd(x, wq, bq, 0.25, bfh, win_pat, qkv, out, lse, n_win, n, nH, win_order=order))
        tg = timeit(lambda: K.linear(x, wq, bq, out=qkv, scale_cols=C, scale_val=0.25))
        fq = 2.0 * n_win * n * C * 3 * C + 4.0 * n * n * hd * n_win * nH
        print(f"win {n_win:5d} heads {nH:3d}: fused qkv+attn {tq * 1e3:7.1f} us {fq / tq / 1e9:6.1f} TF/s   "
              f"(unfused: qkv GEMM {tg * 1e3:6.1f} us + attn {tf * 1e3:6.1f} us)", flush=True)
        tb = 1e-9 if os.environ.get("WATTN_FWD_ONLY") else \
            timeit(lambda: K.wattn_bwd(qkv, out, dout, lse, bbh, win_pat, dqkv, dbp, n_win, n, nH, win))
        if os.environ.get("WATTN_NOBINS"):
            tnb = timeit(lambda: K.wattn_bwd(qkv, out, dout, lse, bbh, win_pat, dqkv, None, n_win, n, nH, win))
            tf32 = timeit(lambda: K.wattn_bwd(qkv, out, dout, lse, bb_, win_pat, dqkv, dbp, n_win, n, nH, win))
            print(f"  bwd with f32 bias tiles {tf32 * 1e3:7.1f} us", flush=True)
            print(f"  bwd without the bias-gradient bins {tnb * 1e3:7.1f} us", flush=True)
        ff, fb = 4.0 * n * n * hd * n_win * nH, 8.0 * n * n * hd * n_win * nH
        tot_f += tf; tot_b += tb; fl_f += ff; fl_b += fb
        print(f"win {n_win:5d} heads {nH:3d}: fwd {tf * 1e3:7.1f} us {ff / tf / 1e9:6.1f} TF/s   "
              f"bwd {tb * 1e3:7.1f} us {fb / tb / 1e9:6.1f} TF/s", flush=True)
    print(f"all stages: fwd {tot_f * 1e3:.1f} us {fl_f / tot_f / 1e9:.1f} TF/s ({fl_f / tot_f / 1e9 / 2500:.3f} of peak)  "
          f"bwd {tot_b * 1e3:.1f} us {fl_b / tot_b / 1e9:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
