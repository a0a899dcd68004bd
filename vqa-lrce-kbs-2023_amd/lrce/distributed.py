"""Data-parallel gradient reduction over RCCL (torch.distributed "nccl" backend on ROCm) / gloo.

Replaces the reference's DDP wrapper (agent_base.py:75-76, train_ddp.py:10-13): one process per
GPU, same model replica, rank-strided batches, gradients averaged every step.  Differences:
* gradients live in ONE flat f32 buffer (lrce/flat.py) laid out in reverse forward order, cut into
  ~bucket_mb contiguous buckets; each native autograd Function reports the parameters it finished,
  and a bucket's all-reduce is launched (async, on RCCL's stream) the moment its last parameter is
  done — so the reduction of the fusion/BERT/late-Swin buckets overlaps the rest of the backward;
* no per-forward buffer broadcast (DDP's broadcast_buffers): the only buffers are constant index
  tables;
* the 1/world average is folded into the optimizer kernel's grad_scale (no extra pass).
Parameters no Function reports (the unused BERT pooler) sit in the last bucket, reduced by finish().
"""
import torch
import torch.distributed as dist


class GradReducer:
    def __init__(self, flat, group=None, bucket_mb=64):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        lim = int(bucket_mb * (1 << 20) // 4)
        self.buckets = []          # (start, end, [param ids])
        self.param_bucket = {}
        cur, start, end = [], None, None
        for p in flat.params:
            s, e = flat.range_of(p)
            if start is None:
                start = s
            cur.append(id(p))
            end = e
            if end - start >= lim:
                self.buckets.append((start, end, cur))
                cur, start = [], None
        if cur:
            self.buckets.append((start, end, cur))
        for bi, (_, _, ids) in enumerate(self.buckets):
            for i in ids:
                self.param_bucket[i] = bi
        self.begin()

    def begin(self):
        self.pending = [len(ids) for _, _, ids in self.buckets]
        self.done = set()
        self.launched = [False] * len(self.buckets)
        self.handles = []

    def _launch(self, bi):
        if self.launched[bi]:
            return
        self.launched[bi] = True
        if self.world > 1:
            s, e, _ = self.buckets[bi]
            self.handles.append(dist.all_reduce(self.flat.grad[s:e], group=self.group, async_op=True))

    def notify(self, params):
        for p in params:
            k = id(p)
            if k in self.done or k not in self.param_bucket:
                continue
            self.done.add(k)
            bi = self.param_bucket[k]
            self.pending[bi] -= 1
            if self.pending[bi] == 0:
                self._launch(bi)

    def finish(self):
        """Launch the remaining buckets (in index order: identical on every rank) and wait for all."""
        for bi in range(len(self.buckets)):
            self._launch(bi)
        for h in self.handles:
            h.wait()
        self.begin()
        return 1.0 / self.world


    def reduce_all(self):
        """All buckets now (graph mode: the backward ran inside a HIP graph with no reducer attached);
        async per bucket on RCCL's stream, then wait.  Returns the optimizer's grad_scale."""
        self.begin()
        return self.finish()


def broadcast_parameters(flat, src=0, group=None):
    """One collective for all 312 M parameters (DDP construction broadcast, agent_base.py:76)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat.f32, src, group=group)
        flat.refresh_bf16()


def attach(model, group=None, bucket_mb=64):
    from .runtime import ensure
    flat = ensure(model)
    red = GradReducer(flat, group, bucket_mb)
    flat.reducer = red
    broadcast_parameters(flat, 0, group)
    return red
