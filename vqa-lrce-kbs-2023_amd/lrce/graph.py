"""HIP-graph capture of a whole training step (the MI355X replacement for a tracing compiler).

A training step of this model issues a few thousand native launches (24 Swin blocks, 12 BERT layers,
3 x 12 recurrent decoder layer-steps, their backward, the fused optimizer).  Issued from Python each
costs host time; captured once into a HIP graph (torch.cuda.CUDAGraph over the same HIP stream the
native kernels launch on) a replay costs one launch.  Everything a step needs is graph-safe:
allocations come from the graph's private pool, dropout masks use seed + a device offset advanced by
a captured add (kernels.rng_advance), DropPath uses torch's graph-aware Philox, and the optimizer's
bias corrections read a device step counter.  Inputs are static buffers: copy a new batch into
`static_inputs` before `replay()` when training on real data.
"""
import torch


class CapturedStep:
    def __init__(self, fn, warmup=2, pool=None):
        """fn(): one training step on the current stream, returning a tensor (e.g. the loss)."""
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
        torch.cuda.synchronize()

    def replay(self):
        self.graph.replay()
        return self.out
