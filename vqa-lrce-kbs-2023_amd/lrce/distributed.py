"""Data-parallel gradient reduction over RCCL (torch.distributed "nccl" backend on ROCm) / gloo.

Replaces the reference's DDP wrapper (agent_base.py:75-76, train_ddp.py:10-13): one process per
GPU, same model replica, rank-strided batches, gradients averaged every step.  Differences:
* gradients live in ONE flat f32 buffer (lrce/flat.py) laid out in reverse forward order, cut into
  ~bucket_mb contiguous buckets; each native autograd Function reports the parameters it finished,
  and a bucket's all-reduce is started the moment its last parameter is done — so the reduction of
  the fusion / BERT / late-Swin buckets overlaps the rest of the backward;
* optional bf16 transport (grad_dtype=torch.bfloat16): the finished bucket is cast once into a bf16
  mirror of the gradient buffer and exchanged as an all-to-all of bf16 shards -> a native f32 sum of
  the world's copies of this rank's shard (lrce_sum_shards_bf16) -> an all-gather of the bf16 sums:
  the same bytes on the xGMI links as a bf16 ring all-reduce (2 (N-1)/N of 0.62 GB instead of 1.25
  GB per step), but the cross-rank sum is f32 (the reference's DDP sums f32), rounded to bf16 once;
  the fused AdamW kernel then reads the bf16 sum directly.  The three steps of a bucket run on a
  communication stream, so the backward on the compute stream never waits for them;
* HIP-graph mode: when the backward is captured into a graph, a finished bucket's bf16 cast is
  captured with it and the bucket is remembered in completion order; after a replay `exchange()`
  issues those buckets' exchanges in that order on the comm stream and the optimizer graph waits
  for them (join()).  torch on ROCm refuses events recorded inside a graph for use outside it
  ("External events are disallowed in rocm", measured on the MI355X box), so the overlap with the
  backward comes from splitting it: TrainStepGraph(tail=model.backward_extractors) captures the
  fusion head's backward and the extractors' backward as two graphs, and the head's buckets (the
  decoder + heads: 115 M of the 312 M parameters) are exchanged while the second graph replays;
  eager mode overlaps every bucket;
* no per-forward buffer broadcast (DDP's broadcast_buffers): the only buffers are constant index
  tables;
* the 1/world average is folded into the optimizer kernel's grad_scale (no extra pass).
Parameters no Function reports (the unused BERT pooler) sit in the last bucket, reduced by finish().
Collectives are issued in bucket-completion order, which is the same on every rank (the backward
is deterministic), as RCCL requires.
"""
import contextlib

import torch
import torch.distributed as dist

from . import kernels as K


def _nullctx():
    return contextlib.nullcontext()


class GradReducer:
    def __init__(self, flat, group=None, bucket_mb=64, grad_dtype=torch.float32):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if grad_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("gradient buckets are f32 or bf16")
        self.grad_dtype = grad_dtype
        # the reduced gradient the optimizer reads (f32: flat.grad itself)
        self.grad16 = torch.zeros(flat.total, dtype=torch.bfloat16, device=flat.device) \
            if grad_dtype == torch.bfloat16 else None
        self.comm = torch.cuda.Stream(device=flat.device) if flat.device.type == "cuda" else None
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
        # bf16 exchange scratch: the all-to-all receive buffer (world shards of the largest bucket) and
        # this rank's summed shard; one each, the buckets' exchanges are ordered on the comm stream
        self.recv = self.shard = None
        if self.grad16 is not None and self.world > 1:
            big = max(e - s for s, e, _ in self.buckets)
            self.recv = torch.empty(big, dtype=torch.bfloat16, device=flat.device)
            self.shard = torch.empty(-(-big // self.world), dtype=torch.bfloat16, device=flat.device)
        self.capturing = False
        self.captured = None       # buckets in completion order (graph mode)
        # test hook: exchange every bf16 bucket by the plain all-reduce fallback (the path a bucket that
        # does not split into 16-B-aligned shards takes)
        self.force_plain = False
        self.begin()

    # ------------------------------------------------------------------ bucket state
    def begin(self):
        self.pending = [len(ids) for _, _, ids in self.buckets]
        self.done = set()
        self.launched = [False] * len(self.buckets)
        self.handles = []
        self.streams = [set() for _ in self.buckets]   # streams whose kernels wrote each bucket

    def reduced_grad(self):
        """The tensor the optimizer reads as the (summed) gradient: flat.grad, or its bf16 mirror."""
        return self.grad16 if self.grad16 is not None else self.flat.grad

    def _buf(self, bi):
        s, e, _ = self.buckets[bi]
        return self.grad16[s:e] if self.grad16 is not None else self.flat.grad[s:e]

    def _launch(self, bi):
        if self.launched[bi]:
            return
        self.launched[bi] = True
        s, e, _ = self.buckets[bi]
        # a bucket straddling the text (side stream) and video / fusion branches: the stream that
        # completes it waits for the other writers before the cast / all-reduce reads it
        if self.flat.grad.is_cuda:
            cur = torch.cuda.current_stream(self.flat.grad.device)
            for st in self.streams[bi]:
                if st != cur:
                    cur.wait_stream(st)
        if self.grad16 is not None:
            K.cast_bf16(self.flat.grad[s:e], self.grad16[s:e])
        if self.capturing:
            self.captured.append(bi)
        elif self.world > 1:
            self._exchange(bi)

    def _exchange(self, bi):
        """Sum bucket bi over the ranks, asynchronously w.r.t. the current (compute) stream.  f32: one
        all-reduce.  bf16: all-to-all of bf16 shards, f32 sum of this rank's shard, all-gather — on the
        comm stream (after the current stream's work so far), which finish() joins."""
        s, e, _ = self.buckets[bi]
        if self.grad16 is None:
            self.handles.append(dist.all_reduce(self.flat.grad[s:e], group=self.group, async_op=True))
            return
        n, w = e - s, self.world
        if n % (8 * w) or self.force_plain:
            # a bucket that does not split into 16-B-aligned shards (only with an odd world size):
            # plain bf16 all-reduce of that bucket
            self.handles.append(dist.all_reduce(self.grad16[s:e], group=self.group, async_op=True))
            return
        sh = n // w
        if self.comm is not None:
            self.comm.wait_stream(torch.cuda.current_stream(self.flat.device))
            ctx = torch.cuda.stream(self.comm)
        else:
            ctx = _nullctx()
        with ctx:
            recv = self.recv[:n]
            dist.all_to_all_single(recv, self.grad16[s:e], group=self.group)
            K.sum_shards_bf16(recv, w, self.shard[:sh])
            dist.all_gather_into_tensor(self.grad16[s:e], self.shard[:sh], group=self.group)

    def _join(self):
        """The current stream waits for every exchange issued so far."""
        for h in self.handles:
            h.wait()
        self.handles = []
        if self.comm is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.comm)

    def notify(self, params):
        cur = torch.cuda.current_stream(self.flat.grad.device) if self.flat.grad.is_cuda else None
        for p in params:
            k = id(p)
            if k in self.done or k not in self.param_bucket:
                continue
            self.done.add(k)
            bi = self.param_bucket[k]
            if cur is not None:
                self.streams[bi].add(cur)
            self.pending[bi] -= 1
            if self.pending[bi] == 0:
                self._launch(bi)

    def finish(self):
        """Launch the remaining buckets (in index order: identical on every rank) and make the
        current stream wait for every all-reduce.  Returns the optimizer's grad_scale (1/world)."""
        for bi in range(len(self.buckets)):
            self._launch(bi)
        if self.capturing:
            return 1.0 / self.world
        self._join()
        self.begin()
        return 1.0 / self.world

    def reduce_all(self):
        """All buckets now (the backward ran with no reducer attached); async per bucket on the
        collective stream, then wait.  Returns the optimizer's grad_scale."""
        self.begin()
        return self.finish()

    # ------------------------------------------------------------------ HIP-graph mode
    def capture_begin(self):
        """Called right before the backward is captured: a bucket completion becomes its captured
        bf16 cast and an entry of the replay order."""
        self.begin()
        self.capturing = True
        self.captured = []

    def capture_end(self):
        self.capturing = False
        self.begin()

    def capture_mark(self):
        """Number of buckets whose completion (bf16 cast) has been captured so far: the split point
        between two captured backward segments (TrainStepGraph with a tail)."""
        return len(self.captured)

    def exchange(self, order):
        """Replay mode: start the exchange of `order`'s buckets (identical on every rank), after the
        current stream's work so far; asynchronous w.r.t. it until join()."""
        if self.world > 1:
            for bi in order:
                self._exchange(bi)

    def chunk_ranges(self, order):
        """The optimizer chunk ranges (1024 elements each; every tensor starts on a chunk) covered by
        the buckets of `order`, merged.  A bucket ends inside its last tensor's final chunk, which no
        other tensor shares, so the ranges of different buckets never overlap."""
        rs = sorted((s // 1024, -(-e // 1024)) for s, e, _ in (self.buckets[bi] for bi in order))
        out = []
        for c0, c1 in rs:
            if out and c0 <= out[-1][1]:
                out[-1] = (out[-1][0], max(out[-1][1], c1))
            else:
                out.append((c0, c1))
        return out

    def exchanged_stream(self):
        """A stream ordered after every exchange started so far, for work that consumes the summed
        buckets while the compute stream moves on: the collective stream, made to wait for the compute
        stream's work so far (the backward that wrote the buckets, whatever path their exchange took)
        and for every async all-reduce handle (f32 buckets and bf16 buckets on the plain all-reduce
        fallback, which run on the process group's own stream).  None on CPU."""
        if self.comm is None:
            return None
        self.comm.wait_stream(torch.cuda.current_stream(self.flat.device))
        with torch.cuda.stream(self.comm):
            for h in self.handles:
                h.wait()
        return self.comm

    def join(self):
        """The current stream waits for every exchange started so far.  Returns the grad_scale."""
        if self.world > 1:
            self._join()
        return 1.0 / self.world

    def replay_allreduce(self, order=None):
        """After replaying the captured backward: one async all-reduce per bucket in capture order
        (identical on every rank), then the current stream waits for all of them (the optimizer
        graph follows).  Returns the optimizer's grad_scale."""
        order = self.captured if order is None else order
        if order is None:
            raise RuntimeError("replay_allreduce: no captured backward")
        self.exchange(order)
        return self.join()


def broadcast_parameters(flat, src=0, group=None):
    """One collective for all 312 M parameters (DDP construction broadcast, agent_base.py:76)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat.f32, src, group=group)
        # the collective writes the masters without bumping any tensor version counter: re-cast the
        # bf16 / fp16 shadows unconditionally and invalidate the optimizer's norm cache
        flat.masters_written()


def attach(model, group=None, bucket_mb=64, grad_dtype=torch.float32):
    from .runtime import ensure
    flat = ensure(model)
    red = GradReducer(flat, group, bucket_mb, grad_dtype)
    flat.reducer = red          # notify target of the native backward Functions (may be detached)
    flat.grad_reducer = red     # the optimizer reads red.reduced_grad()
    broadcast_parameters(flat, 0, group)
    return red
