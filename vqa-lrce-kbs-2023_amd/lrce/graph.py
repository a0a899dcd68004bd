"""HIP-graph capture of a whole training step (the MI355X replacement for a tracing compiler).

A training step of this model issues a few thousand native launches (24 Swin blocks, 12 BERT layers,
3 x 12 recurrent decoder layer-steps, their backward, the fused optimizer).  Issued from Python each
costs host time; captured once into a HIP graph (torch.cuda.CUDAGraph over the same HIP stream the
native kernels launch on) a replay costs one launch.  Everything a step needs is graph-safe:
allocations come from the graph's private pool, dropout masks use seed + a device offset advanced by
a captured add (kernels.rng_advance), DropPath uses torch's graph-aware Philox, the optimizer's
bias corrections read a device step counter and its learning rates a device table refreshed before
each replay.  Inputs are static buffers: TrainStepGraph copies each batch into them.
"""
import os

import torch

from .runtime import join_capture_branches

# HIP runtime debug variable that hands a graph's parallel branches to N extra queues.  With it set to
# 8 the ROCm 7 runtime crashed in the first captured training step of this model (round-4 A/B variant
# "fq8": core dump at the capture; reproduced once in round 5: segmentation fault), so the capture
# refuses it with an explanation instead of reaching that crash.  The round-5 crash (A/B "r5ab2", a
# SIGSEGV in the first captured step after half of BERT's weight-gradient flush moved to a new sixth
# stream) shares the trait of one more stream branch in the graph; its diff was reverted before a
# commit, so the exact fault is not reconstructible.  The capture therefore refuses the patterns that
# trait can take (runtime.aux_stream): a branch name outside the captured-and-replayed set, and a
# stream created while capturing; and it joins every branch forked into a capture back into the
# capturing stream before the capture ends (runtime.join_capture_branches), so an unjoined fork can
# never reach the runtime's end-of-capture path.
_FORCE_GRAPH_QUEUES = "DEBUG_HIP_FORCE_GRAPH_QUEUES"


def _check_runtime_env():
    v = os.environ.get(_FORCE_GRAPH_QUEUES, "")
    if v not in ("", "0"):
        raise RuntimeError(f"{_FORCE_GRAPH_QUEUES}={v} is set: the HIP runtime crashes replaying this model's "
                           f"captured training step under that debug setting (DESIGN.md §8); unset it")


class CapturedStep:
    def __init__(self, fn, warmup=2, pool=None):
        """fn(): one training step on the current stream, returning a tensor (e.g. the loss)."""
        _check_runtime_env()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=pool):
            self.out = fn()
            join_capture_branches(torch.cuda.current_stream().device)
        torch.cuda.synchronize()

    def replay(self):
        self.graph.replay()
        return self.out


class _Captured:
    __slots__ = ("static", "out", "g_step", "g_tail", "g_opt", "g_early", "warm", "order", "order_tail", "stage", "turn",
                 "free")
    # g_tail / order_tail: one captured graph and one bucket-order list per tail segment; g_early: the
    # optimizer update of the buckets exchanged before each tail segment (None: not split)

    def __init__(self, inputs, device):
        self.static = [torch.empty_like(t, device=device) for t in inputs]
        self.out = self.g_step = self.g_tail = self.g_opt = self.g_early = self.order = self.order_tail = None
        self.warm = False
        # two device staging sets for host batches: the H2D copy of batch i+1 runs on a side stream
        # while step i is still replaying, and never overwrites a set the main stream still reads
        self.stage = [[torch.empty_like(t, device=device) for t in inputs] for _ in range(2)] \
            if any(not t.is_cuda for t in inputs) else None
        self.turn = 0
        self.free = [None, None]   # main-stream events: staging set k has been copied out


class TrainStepGraph:
    """The agent's training step (agent_oe.py:19-48 and its MC / count twins) replayed from HIP
    graphs: forward -> task loss -> backward [-> all-reduce of the gradient buckets] -> fused AdamW.

    body(*static_inputs) runs forward + loss + backward and returns the tensors the caller reads
    (logits, per-sample loss terms, ...).  On one rank the optimizer step is captured into the same
    graph; with a GradReducer (world > 1) the step is graph(forward + backward, with the bf16 bucket
    casts) -> the bucket all-reduces in capture order -> graph(optimizer).  The first call with a
    new input signature (shapes / dtypes) runs the step eagerly (allocator / kernel warm-up, a real
    training step) and captures on the next one; graphs are kept per signature (a short last batch
    gets its own).  Every call is exactly one training step.

    tail (optional, with a reducer): the rest of a split backward (E2EBase.split_backward), one callable
    or a list of segments (E2EBase.backward_segments): body then ends with the fusion head's backward,
    and the step is graph(forward + head backward) -> exchange of the head's buckets, overlapping ->
    graph(segment 1) -> exchange of the buckets it completed, overlapping -> graph(segment 2) ... ->
    exchange of the rest -> graph(optimizer).

    early_opt (with a tail): the optimizer update of the buckets exchanged before a segment (the head's
    before segment 1, segment 1's before segment 2, ...) is captured as a graph of its own and replayed
    on the collective stream right behind that exchange, so it runs beside the next backward segment
    (which reads none of those parameters) instead of after the whole backward; the final optimizer
    graph updates the rest and sums the next step's norms (agent_base.py:76's DDP overlap, carried
    through to the update)."""

    def __init__(self, body, optim, reducer=None, world=1, tail=None, early_opt=True):
        self.body, self.optim, self.reducer, self.world = body, optim, reducer, world
        self.early_opt = early_opt
        if tail is not None and not isinstance(tail, (list, tuple)):
            tail = [tail]
        self.tail = list(tail) if (tail and reducer is not None) else None
        self.states = {}
        self.static = None   # static inputs of the last call (the agent reads the labels from it)
        self.copy_stream = None
        # ONE private memory pool for every signature's graphs: a short last batch captured into a pool
        # of its own would keep a second step's activations resident.  Sharing is safe here because
        # no two graphs ever replay concurrently and a graph's outputs are read only right after its
        # own replay (the blocks another signature's capture reused hold only that graph's temporaries).
        self.pool = None

    def _load(self, st, inputs):
        """Batch -> the static input buffers.  Host tensors (pinned by the DataLoader) go H2D on a
        side stream into a staging set, overlapping the previous step's replay; the main stream
        then waits for that copy and moves the batch with a device-to-device copy."""
        cur = torch.cuda.current_stream(self.optim.flat.device)
        if st.stage is None:
            for s, t in zip(st.static, inputs):
                s.copy_(t, non_blocking=True)
            return
        if self.copy_stream is None:
            self.copy_stream = torch.cuda.Stream(self.optim.flat.device)
        k = st.turn
        st.turn ^= 1
        stage = st.stage[k]
        cs = self.copy_stream
        if st.free[k] is not None:
            cs.wait_event(st.free[k])          # the main stream has moved this set's last batch out
        with torch.cuda.stream(cs):
            for d, t in zip(stage, inputs):
                d.copy_(t, non_blocking=True)
        cur.wait_event(cs.record_event())
        for s, d in zip(st.static, stage):
            s.copy_(d, non_blocking=True)
        st.free[k] = cur.record_event()

    @staticmethod
    def _sig(inputs):
        return tuple((tuple(t.shape), t.dtype) for t in inputs)

    def _eager(self, st):
        st.out = self.body(*st.static)
        for seg in self.tail or ():
            seg()
        scale = self.reducer.finish() if self.reducer is not None else 1.0
        self.optim.step(grad_scale=scale)
        return st.out

    def _capture(self, st):
        _check_runtime_env()
        torch.cuda.synchronize()
        self.optim._sync_lrs()          # no host->device copy may land inside the capture
        steps = self.optim.step_count   # the host-side count of a captured step() is not a real step
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        pool = self.pool
        st.g_step = torch.cuda.CUDAGraph()
        if self.reducer is None:
            with torch.cuda.graph(st.g_step, pool=pool):
                st.out = self.body(*st.static)
                self.optim.step(grad_scale=1.0)
                join_capture_branches(self.optim.flat.device)
        else:
            self.reducer.capture_begin()
            try:
                if self.tail is None:
                    with torch.cuda.graph(st.g_step, pool=pool):
                        st.out = self.body(*st.static)
                        self.reducer.finish()            # captures the remaining buckets' bf16 casts
                        join_capture_branches(self.optim.flat.device)
                    st.order = list(self.reducer.captured)
                else:
                    with torch.cuda.graph(st.g_step, pool=pool):
                        st.out = self.body(*st.static)
                        if self.early_opt:
                            # the step's optimizer bookkeeping (device step counter, lr table, a norm
                            # pass if the masters changed outside the optimizer) on the main stream,
                            # ahead of every exchange: the early-update graphs then hold only updates
                            self.optim._begin()
                        join_capture_branches(self.optim.flat.device)
                    marks = [self.reducer.capture_mark()]
                    st.g_tail = []
                    for i, seg in enumerate(self.tail):
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g, pool=pool):
                            seg()
                            if i == len(self.tail) - 1:
                                self.reducer.finish()
                            join_capture_branches(self.optim.flat.device)
                        st.g_tail.append(g)
                        marks.append(self.reducer.capture_mark())
                    st.order = list(self.reducer.captured[:marks[0]])
                    st.order_tail = [list(self.reducer.captured[a:b]) for a, b in zip(marks[:-1], marks[1:])]
            finally:
                self.reducer.capture_end()
            if self.tail is not None and self.early_opt:
                # one update graph per exchange that a later segment overlaps; its own memory pool,
                # since it replays concurrently with a backward segment (it allocates nothing anyway)
                epool = torch.cuda.graph_pool_handle()
                st.g_early = []
                for order in [st.order] + st.order_tail[:-1]:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=epool):
                        self.optim.update_chunks(self.reducer.chunk_ranges(order), grad_scale=1.0 / self.world)
                        join_capture_branches(self.optim.flat.device)
                    st.g_early.append(g)
            st.g_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(st.g_opt, pool=pool):
                self.optim.step(grad_scale=1.0 / self.world)
                join_capture_branches(self.optim.flat.device)
        self.optim.step_count = steps
        self.optim.flat.mark_bf16_fresh()
        torch.cuda.synchronize()

    def __call__(self, *inputs):
        key = self._sig(inputs)
        st = self.states.get(key)
        if st is None:
            st = self.states[key] = _Captured(inputs, self.optim.flat.device)
        self.static = st.static
        self._load(st, inputs)
        if not st.warm:
            st.warm = True
            return self._eager(st)
        if st.g_step is None:
            try:
                self._capture(st)
            except BaseException:
                # a failed capture must not leave the optimizer believing this step has begun (the next
                # eager step would skip its step-counter increment) or that chunks were updated
                self.optim._begun = False
                self.optim._done = []
                st.g_step = None
                raise
        self.optim._sync_lrs()
        st.g_step.replay()
        if st.g_tail is not None:
            self.reducer.exchange(st.order)        # the head's buckets, beside the extractors' backward
            for i, (g, order) in enumerate(zip(st.g_tail, st.order_tail)):
                if st.g_early is not None:         # their update too, behind the exchange
                    with torch.cuda.stream(self.reducer.exchanged_stream()):
                        st.g_early[i].replay()
                g.replay()
                self.reducer.exchange(order)       # this segment's buckets, beside the next segment
            self.reducer.join()
            st.g_opt.replay()
        elif st.g_opt is not None:
            self.reducer.replay_allreduce(st.order)
            st.g_opt.replay()
        self.optim.step_count += 1      # host bookkeeping the captured optimizer step cannot do
        return st.out
