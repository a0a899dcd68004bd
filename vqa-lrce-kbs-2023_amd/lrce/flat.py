"""Flat parameter storage for a module on one HIP device.

All parameters live as views of ONE f32 master buffer; a bf16 shadow of the same layout feeds the
MFMA kernels; gradients are views of ONE f32 buffer that the backward kernels accumulate into
directly (atomics / fused epilogues), so there is no per-parameter autograd accumulation pass.
Every tensor starts on a 1024-element boundary, so 1024-element chunks map to exactly one tensor:
this is what lets the fused L2-norm + AdamW kernels (csrc/optim.hip) and the gradient all-reduce
buckets work on plain contiguous ranges.  Parameter names/shapes are untouched, so state_dict()
keeps the reference key schema.
"""
import torch

from . import kernels as K

ALIGN = 1024


class FlatParams:
    def __init__(self, module, device, order=None):
        self.device = torch.device(device)
        self.params = [p for p in module.parameters()]
        if order is not None:  # layout order (e.g. reverse forward order for gradient buckets)
            ids = {id(p) for p in self.params}
            assert len(order) == len(self.params) and {id(p) for p in order} == ids, "order must permute parameters"
            self.params = list(order)
        self.reducer = None          # notify target during a backward (lrce/distributed.py)
        self.early_update = None     # optimizer hook: a parameter group's gradients are final (optim.py)
        self.step_begin_hook = None  # optimizer hook: a training forward starts (optim.py)
        self.grad_reducer = None     # its GradReducer, whose reduced gradient the optimizer reads
        self.names = {id(p): n for n, p in module.named_parameters()}
        offs, o = [], 0
        for p in self.params:
            offs.append(o)
            o += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.total = o
        self.offsets = offs
        self.f32 = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.bf16 = torch.empty(self.total, dtype=torch.bfloat16, device=self.device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self._index = {}
        for i, (p, off) in enumerate(zip(self.params, offs)):
            n = p.numel()
            self.f32[off:off + n].copy_(p.detach().reshape(-1))
            p.data = self.f32[off:off + n].view(p.shape)
            self._index[id(p)] = i
        chunk_tensor = torch.empty(self.total // ALIGN, dtype=torch.int32)
        for i, (p, off) in enumerate(zip(self.params, offs)):
            n = (p.numel() + ALIGN - 1) // ALIGN
            chunk_tensor[off // ALIGN: off // ALIGN + n] = i
        self.chunk_tensor = chunk_tensor.to(self.device)
        self.n_chunks = self.total // ALIGN
        # first chunk of every tensor (+ end): the deterministic per-tensor norm sums (csrc/optim.hip)
        off = torch.tensor([o // ALIGN for o in offs] + [self.n_chunks], dtype=torch.int32)
        self.tensor_chunk_off = off.to(self.device)
        self._bf16_version = -1
        self._epoch = 0            # bumped by writes the version counters cannot see (collectives)
        # gradient freshness (claim_fresh): generation of the last optimizer zero_grad, and per
        # parameter the generation its gradient was last claimed in
        self._zero_gen = 0
        self._claimed = {}
        self.f16 = None            # optional IEEE fp16 shadow of [f16_lo, f16_hi) (enable_f16)
        self.f16_lo = self.f16_hi = 0
        self.attach_grads(zero=True)

    def enable_f16(self, params):
        """Keep an fp16 shadow of the flat range spanning `params` (the BERT weights: its forward
        runs in fp16 like the reference's autocast).  The optimizer refreshes it with the bf16 one."""
        params = [p for p in params if self.owns(p)]
        if not params:
            return
        lo = min(self.range_of(p)[0] for p in params)
        hi = max(self.range_of(p)[1] for p in params)
        self.f16_lo, self.f16_hi = lo, hi
        self.f16 = torch.empty(hi - lo, dtype=torch.float16, device=self.device)
        K.cast_f16(self.f16_src(), self.f16)
        self._bf16_version = -1

    def f16_src(self):
        return self.f32[self.f16_lo:self.f16_hi]

    def has_f16(self, p):
        """Does the fp16 shadow cover p?"""
        if self.f16 is None or id(p) not in self._index:
            return False
        off = self.offsets[self._index[id(p)]]
        return self.f16_lo <= off and off + p.numel() <= self.f16_hi

    def w16h(self, p):
        """fp16 shadow of p (enable_f16 must cover it)."""
        i = self._index[id(p)]
        off = self.offsets[i] - self.f16_lo
        if self.f16 is None or off < 0 or off + p.numel() > self.f16.numel():
            raise RuntimeError(f"no fp16 shadow for {self.names.get(id(p), '?')}: call enable_f16 first")
        return self.f16[off:off + p.numel()].view(p.shape)

    def grads_zeroed(self):
        """The optimizer has just cleared every gradient (FusedAdamW.zero_grad)."""
        self._zero_gen += 1

    def claim_fresh(self, params):
        """True iff no gradient of `params` has been claimed since the last optimizer zero_grad — a
        weight-gradient GEMM may then STORE its product instead of adding it to the (zero) gradient
        (half the epilogue's memory traffic, no read round trip).  Claims them either way, so a second
        backward before the next zero_grad accumulates.  False whenever the gradients were cleared
        some other way (attach_grads, set_to_none): the accumulating path is always correct."""
        g = self._zero_gen
        fresh = g > 0 and all(self._claimed.get(id(p), 0) != g for p in params)
        for p in params:
            self._claimed[id(p)] = g
        return fresh

    def notify(self, params):
        """Called by native autograd Functions when their parameters' gradients are final."""
        if self.reducer is not None:
            self.reducer.notify(params)

    def step_begin(self):
        """A training forward starts (on the stream the step's other streams fork from)."""
        if self.step_begin_hook is not None:
            self.step_begin_hook()

    def group_done(self, name):
        """A whole parameter group's gradients are final (on the current stream): the optimizer may
        update that group now, off the critical path (FusedAdamW.enable_early_updates)."""
        if self.early_update is not None:
            self.early_update(name)

    def chunk_range(self, params):
        """[c0, c1) in 1024-element chunks covering exactly `params` (they must be contiguous in the
        layout: no other parameter inside)."""
        idx = sorted(self._index[id(p)] for p in params)
        if not idx or idx != list(range(idx[0], idx[-1] + 1)):
            raise ValueError("parameters are not contiguous in the flat layout")
        return self.offsets[idx[0]] // ALIGN, self.range_of(self.params[idx[-1]])[1] // ALIGN

    # ------------------------------------------------------------------ views
    def _slice(self, buf, p):
        i = self._index[id(p)]
        off = self.offsets[i]
        return buf[off:off + p.numel()].view(p.shape)

    def w16(self, p):
        return self._slice(self.bf16, p)

    def g32(self, p):
        """f32 gradient accumulator of p (None if p is frozen)."""
        if not p.requires_grad:
            return None
        return self._slice(self.grad, p)

    def range_of(self, p):
        i = self._index[id(p)]
        return self.offsets[i], self.offsets[i] + (p.numel() + ALIGN - 1) // ALIGN * ALIGN

    def owns(self, p):
        return id(p) in self._index

    # ------------------------------------------------------------------ sync
    def _versions(self):
        """(version of the f32 buffer, sum of the parameters' own version counters).  Writes through
        slices of f32 bump the first; in-place writes through a parameter (load_state_dict's copy_,
        `p.mul_()` under no_grad) bump only that parameter's counter, because `p.data = view` keeps
        the parameter's own counter — hence both."""
        return self.f32._version, sum(p._version for p in self.params), self._epoch

    def refresh_bf16(self):
        """Re-cast the bf16 shadow if the masters changed (optimizer step, load_state_dict, ...)."""
        v = self._versions()
        if v != self._bf16_version:
            K.cast_bf16(self.f32, self.bf16)
            if self.f16 is not None:
                K.cast_f16(self.f16_src(), self.f16)
            self._bf16_version = self._versions()

    def masters_written(self):
        """The f32 masters were overwritten behind torch's back (e.g. an in-place broadcast): refresh
        the 16-bit shadows now and invalidate every cache keyed on master_version()."""
        self._epoch += 1
        K.cast_bf16(self.f32, self.bf16)
        if self.f16 is not None:
            K.cast_f16(self.f16_src(), self.f16)
        self._bf16_version = self._versions()

    def mark_bf16_fresh(self):
        self._bf16_version = self._versions()

    def master_version(self):
        """Changes whenever any master weight changed (the optimizer's norm cache key)."""
        return self._versions()

    def attach_grads(self, zero=False):
        """Make every p.grad the flat view (torch's zero_grad(set_to_none=True) drops them)."""
        need = zero
        for p in (self.params[0], self.params[-1]):  # zero_grad() touches all or none
            if not p.requires_grad:
                continue
            g = p.grad
            if g is None or g.data_ptr() != self._slice(self.grad, p).data_ptr():
                need = True
        if need:
            self.grad.zero_()
            for p in self.params:
                p.grad = self._slice(self.grad, p) if p.requires_grad else None
