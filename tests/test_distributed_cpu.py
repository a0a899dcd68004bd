"""Data-parallel gradient reduction (lrce/distributed.py) with world_size 2 over gloo on CPU.

The reference wraps the model in DDP (agent_base.py:75-76, train_ddp.py:10-13): after backward every
rank holds the average of the ranks' gradients.  Here the flat gradient buffer is cut into buckets
that are all-reduced as soon as their parameters are final (notify) or all at once (reduce_all),
and the 1/world average is returned as the optimizer's grad_scale.  These tests run the real
GradReducer / FlatParams on CPU tensors in two gloo processes (no GPU, no native kernels)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "vqa-lrce-kbs-2023_amd")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Toy(nn.Module):
    """A few parameters of very different sizes (several buckets at a 1 MB bucket limit)."""

    def __init__(self):
        super().__init__()
        self.a = nn.Linear(512, 512)       # 262 656 params ~ 1 MB
        self.b = nn.Linear(512, 8)
        self.c = nn.Parameter(torch.zeros(300_000))
        self.d = nn.LayerNorm(64)


def _worker(rank, world, port, mode, q):
    import sys
    sys.path.insert(0, PKG)
    from lrce.distributed import GradReducer
    from lrce.flat import FlatParams
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        model = _Toy()
        flat = FlatParams(model, "cpu", order=list(model.parameters())[::-1])
        if mode == "bf16":
            # the exchange's two native kernels, restated in torch for CPU tensors (test stand-ins:
            # the product raises on CPU tensors)
            from lrce import kernels as K
            K.cast_bf16 = lambda x, y: y.copy_(x.to(torch.bfloat16))
            K.sum_shards_bf16 = lambda src, n, dst: dst.copy_(src.view(n, -1).float().sum(0).to(torch.bfloat16))
            red = GradReducer(flat, bucket_mb=1, grad_dtype=torch.bfloat16)
        else:
            red = GradReducer(flat, bucket_mb=1)
        out = {"n_buckets": len(red.buckets)}
        # rank-specific gradients: g_r = (r + 1) * base
        base = torch.arange(flat.total, dtype=torch.float32) % 97
        flat.grad.copy_(base * (rank + 1))
        if mode in ("notify", "bf16"):
            # report parameters in backward order; buckets launch as they complete
            for p in reversed(list(model.parameters())):
                red.notify([p])
            out["launched_before_finish"] = sum(red.launched)
            scale = red.finish()
        else:
            scale = red.reduce_all()
        out["scale"] = scale
        g = red.reduced_grad().float()
        out["grad_sum"] = g.double().sum().item()
        out["grad_head"] = g[:8].tolist()   # plain data: no shared-memory handle outlives the child
        if mode == "bf16":
            # the f32 sum of the ranks' bf16 copies, rounded once: here exact (small integers)
            ref = ((base * (rank + 1)).to(torch.bfloat16).float() + (base * (2 - rank)).to(torch.bfloat16).float())
            out["bf16_exact"] = bool(torch.equal(g, ref.to(torch.bfloat16).float()))
        out["param_view_is_flat"] = all(p.grad.data_ptr() == flat.g32(p).data_ptr() for p in model.parameters())
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _run(mode, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("mode", ["notify", "reduce_all", "bf16"])
def test_grad_reducer_sums_over_ranks_gloo(mode):
    res = _run(mode)
    r0, r1 = res[0], res[1]
    assert r0["n_buckets"] >= 2                       # bucketing actually splits the flat buffer
    assert r0["scale"] == pytest.approx(0.5) and r1["scale"] == pytest.approx(0.5)
    # all-reduce (sum) of (r+1)*base over 2 ranks = 3*base on both ranks; the optimizer applies 1/world
    assert r0["grad_head"] == r1["grad_head"]
    base_head = torch.arange(8, dtype=torch.float32) % 97
    assert r0["grad_head"] == (3 * base_head).tolist()
    assert r0["grad_sum"] == pytest.approx(r1["grad_sum"])
    assert r0["param_view_is_flat"] and r1["param_view_is_flat"]
    if mode in ("notify", "bf16"):
        assert r0["launched_before_finish"] == r0["n_buckets"]   # every bucket launched from notify()
    if mode == "bf16":
        # bf16 transport (all-to-all, f32 shard sum, all-gather): same sums on every rank
        assert r0["bf16_exact"] and r1["bf16_exact"]


def test_flat_layout_alignment_cpu():
    """Every tensor of the flat store starts on a 1024-element boundary (fused L2/AdamW chunk map)."""
    import sys
    sys.path.insert(0, PKG)
    from lrce.flat import ALIGN, FlatParams
    model = _Toy()
    flat = FlatParams(model, "cpu")
    assert all(o % ALIGN == 0 for o in flat.offsets)
    assert flat.total % ALIGN == 0
    ct = flat.chunk_tensor
    for i, p in enumerate(flat.params):
        s, e = flat.range_of(p)
        assert bool((ct[s // ALIGN:e // ALIGN] == i).all())
