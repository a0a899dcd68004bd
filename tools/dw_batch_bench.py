#!/usr/bin/env python
"""Weight gradients of a Swin stage's blocks (dev tool, GPU): n_blocks separate split-K launches
(linear_dw: f32 slabs + reduce, what the block backward issues) against ONE batched launch over the
blocks (batch = n_blocks, one K slice per tile, ACCUM + BIAS_GRAD with per-batch strides), on the
stage-3 shapes; then a stage's flush as one launch per shape against ONE grouped launch over every
linear and block (stage 3: 18 blocks, stage 4: 2 blocks).  HIP events over back-to-back repetitions.

    python tools/dw_batch_bench.py [--blocks 18] [--iters 5]
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

# (name, out, in): dW[out, in] += dY[T, out]^T X[T, in] over T tokens
SHAPES = [("qkv", 1536, 512), ("proj", 512, 512), ("fc1", 2048, 512), ("fc2", 512, 2048)]


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=18)
    ap.add_argument("--tokens", type=int, default=17640)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    nb, T = a.blocks, a.tokens
    bf = torch.bfloat16
    total_sep = total_bat = 0.0
    for name, O, I in SHAPES:
        dy = torch.rand(nb, T, O, device="cuda").sub_(0.5).to(bf)
        x = torch.rand(nb, T, I, device="cuda").sub_(0.5).to(bf)
        dw = torch.zeros(nb, O, I, device="cuda")
        db = torch.zeros(nb, O, device="cuda")

        def sep():
            for j in range(nb):
                K.linear_dw(dy[j], x[j], dw[j], bias_grad=db[j])

        def bat():
            K.gemm(dy, x, dw, O, I, T, a_kmajor=False, b_kmajor=False, lda=O, ldb=I, ldc=I,
                   flags=N.EPI_ACCUM | N.EPI_BIAS_GRAD, bias=db, batch=nb, stride_a=T * O, stride_b=T * I,
                   stride_c=O * I, stride_bias=O)

        # agreement: both from zero
        dw.zero_(); db.zero_(); sep(); ref_w, ref_b = dw.clone(), db.clone()
        dw.zero_(); db.zero_(); bat()
        err = ((dw - ref_w).abs().max() / ref_w.abs().max()).item()
        errb = ((db - ref_b).abs().max() / ref_b.abs().max()).item()
        ts, tb = timed(sep, a.iters), timed(bat, a.iters)
        total_sep += ts
        total_bat += tb
        fl = 2.0 * nb * T * O * I
        print(f"{name:5s} {O:5d}x{I:5d}x{T}: {nb} split-K launches {ts:8.1f} us ({fl / ts / 1e6:6.1f} TF/s)   "
              f"batched {tb:8.1f} us ({fl / tb / 1e6:6.1f} TF/s)   rel diff w {err:.1e} b {errb:.1e}", flush=True)
    print(f"stage total: separate {total_sep:.1f} us, batched {total_bat:.1f} us")
    grouped_vs_per_shape(nb, T, SHAPES, a.iters)
    C4 = [("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096)]
    grouped_vs_per_shape(2, T // 4, C4, a.iters)
    for C, TT in ((256, T * 4), (128, T * 16)):   # stages 2 and 1: few tiles over a long K
        split_vs_per_item(2, TT, [("qkv", 3 * C, C), ("proj", C, C), ("fc1", 4 * C, C), ("fc2", C, 4 * C)], a.iters)


def split_vs_per_item(nb, T, shapes, iters):
    """A long-K stage's weight gradients: one split-K launch + reduce per linear (linear_dw, the
    immediate path) against ONE grouped launch with per-entry K slices + one slab-sum launch."""
    bf = torch.bfloat16
    items = []
    for j in range(nb):
        for name, O, I in shapes:
            items.append((torch.rand(T, O, device="cuda").sub_(0.5).to(bf), torch.rand(T, I, device="cuda").sub_(0.5).to(bf),
                          torch.zeros(O, I, device="cuda"), torch.zeros(O, device="cuda"), False))
    tiles = sum(-(-O // 128) * -(-I // 128) for _, O, I in shapes) * nb
    split = max(2, min(64, round(512 / tiles)))

    def per_item():
        for dy, x, dw, db, _ in items:
            K.linear_dw(dy, x, dw, bias_grad=db)

    def grouped():
        K.linear_dw_grouped(items, split=split)

    per_item(); torch.cuda.synchronize()
    ref = [(it[2].clone(), it[3].clone()) for it in items]
    for it in items:
        it[2].zero_(); it[3].zero_()
    grouped(); torch.cuda.synchronize()
    err = max(((it[2] - r[0]).abs().max() / r[0].abs().max()).item() for it, r in zip(items, ref))
    errb = max(((it[3] - r[1]).abs().max() / r[1].abs().max()).item() for it, r in zip(items, ref))
    tp, tg = timed(per_item, iters), timed(grouped, iters)
    fl = sum(2.0 * T * O * I for _, O, I in shapes) * nb
    print(f"{nb} blocks x C={shapes[1][1]} T={T} ({tiles} tiles, split {split}): per-item split-K {tp:8.1f} us "
          f"({fl / tp / 1e6:6.1f} TF/s)   grouped split {tg:8.1f} us ({fl / tg / 1e6:6.1f} TF/s)   "
          f"rel diff w {err:.1e} b {errb:.1e}", flush=True)


def grouped_vs_per_shape(nb, T, shapes, iters):
    """A stage's flush: the blocks' weight gradients as one same-shape launch per linear
    (linear_dw_batched) against ONE grouped launch over every linear and block (linear_dw_grouped)."""
    bf = torch.bfloat16
    items = []
    for j in range(nb):
        for name, O, I in shapes:
            items.append((torch.rand(T, O, device="cuda").sub_(0.5).to(bf), torch.rand(T, I, device="cuda").sub_(0.5).to(bf),
                          torch.zeros(O, I, device="cuda"), torch.zeros(O, device="cuda"), False))

    def per_shape():
        for k in range(len(shapes)):
            K.linear_dw_batched([it[:4] for it in items[k::len(shapes)]])

    def grouped():
        K.linear_dw_grouped(items)

    per_shape(); torch.cuda.synchronize()
    ref = [(it[2].clone(), it[3].clone()) for it in items]
    for it in items:
        it[2].zero_(); it[3].zero_()
    grouped(); torch.cuda.synchronize()
    err = max(((it[2] - r[0]).abs().max() / r[0].abs().max()).item() for it, r in zip(items, ref))
    tp, tg = timed(per_shape, iters), timed(grouped, iters)
    t2 = timed(lambda: K.linear_dw_grouped(items, split=2), iters)
    fl = sum(2.0 * T * O * I for _, O, I in shapes) * nb
    print(f"{nb} blocks x {[s[0] for s in shapes]} T={T}: per-shape launches {tp:8.1f} us ({fl / tp / 1e6:6.1f} TF/s)   "
          f"grouped {tg:8.1f} us ({fl / tg / 1e6:6.1f} TF/s)   grouped 2 K slices {t2:8.1f} us   "
          f"first-pass rel diff {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
