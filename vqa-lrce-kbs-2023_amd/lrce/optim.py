"""Fused AdamW over the flat parameter store (reference agent_base.py:27-44 + the L2 regulariser of
agent_base.py:103-108 / agent_oe.py:36).

The reference builds torch.optim.AdamW with three parameter groups (fusion, text, video; lr may be
given per group, args.py:110-111) and adds reg_strength * sum_t ||p_t||_2 to the loss, so every
step back-propagates 783 norm kernels.  Here the regulariser's gradient reg * p_t / ||p_t|| is
added inside the update kernel (csrc/optim.hip) from one multi-tensor norm pass: the optimizer step
is two launches for all 312 M parameters, and it also refreshes the bf16 shadow the forward reads.
Semantics = torch.optim.AdamW (decoupled weight decay 0.01 default, bias-corrected moments).
"""

import torch

from . import kernels as K
from .runtime import aux_stream, flat_of, ensure


def guard_skip(guard, c0, c1):
    """The found-inf skip argument of an update over chunks [c0, c1): guard = ((s0, s1), slots) — the
    guarded chunk range and its scale slots — or None.  Returns (slots, first, end) relative to c0 for
    the part of [s0, s1) inside [c0, c1), or None when they do not meet."""
    if guard is None:
        return None
    (s0, s1), slots = guard
    lo, hi = max(s0, c0), min(s1, c1)
    return (slots, lo - c0, hi - c0) if lo < hi else None


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, model, groups, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, reg_strength=0.0):
        """groups: list of iterables of parameters (e.g. [fusion.parameters(), text..., video...]) or of
        dicts {'params': ..., 'lr': ...}; every parameter must belong to `model`'s flat store."""
        flat = flat_of(model) or ensure(model)
        pg = []
        for g in groups:
            if isinstance(g, dict):
                pg.append({"params": list(g["params"]), "lr": g.get("lr", lr)})
            else:
                pg.append({"params": list(g), "lr": lr})
        super().__init__(pg, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.flat = flat
        self.reg_strength = float(reg_strength)
        dev = flat.device
        self.exp_avg = torch.zeros_like(flat.f32)
        self.exp_avg_sq = torch.zeros_like(flat.f32)
        self.sumsq = torch.zeros(len(flat.params), device=dev)        # ||p_t||^2 of the current parameters
        self.sumsq_next = torch.zeros(len(flat.params), device=dev)   # written by the update step
        self.chunk_sq = torch.zeros(flat.n_chunks, device=dev)        # per-chunk sums (deterministic norms)
        self._norm_version = None   # flat.master_version() the norms belong to (None: never computed)
        self._index = {id(p): i for i, p in enumerate(flat.params)}
        self.tensor_lr = torch.zeros(len(flat.params), device=dev)
        self._lr_cache = None
        self.step_count = 0
        self.step_t = torch.zeros(1, device=dev)   # device step count t (graph-safe bias corrections)
        self.last_l2 = None
        self._early = {}        # group name -> chunk range updated as soon as its gradients are final
        self._begun = False     # this step's counters / norms are set up (_begin)
        self._done = []         # chunk ranges already updated this step
        self.early_updates = 0  # group updates issued from inside a backward (statistics)
        # found-inf guard: the chunk range whose gradients come from delayed-scale fp16 operands and those
        # operands' scale slots (model.overflow_guard(): BERT's); an overflow skips that range's update
        guard = getattr(model, "overflow_guard", None)
        self._guard = None
        if guard is not None:
            params, slots = guard(dev)
            self._guard = (flat.chunk_range(params), slots)

    def enable_early_updates(self, groups):
        """groups: {name: parameters}.  When the backward reports a group final (flat.group_done,
        called on the stream that produced its last gradient) that group is updated right there, so
        e.g. the decoder's and BERT's updates overlap the Swin backward instead of following it.
        Single process only: with a gradient reducer the update must wait for the all-reduce."""
        self._early = {name: self.flat.chunk_range(list(ps)) for name, ps in groups.items()}
        self.flat.early_update = self._early_update if self._early else None
        # the step's device bookkeeping (step counter, norms) runs when the training forward starts,
        # on the stream every later stream forks from (E2EBase.forward -> flat.step_begin)
        self.flat.step_begin_hook = self._begin if self._early else None

    def _begin(self):
        if self._begun:
            return
        flat = self.flat
        self._sync_lrs()
        self.step_count += 1
        self.step_t.add_(1.0)
        if self._norm_version != flat.master_version():
            # parameters changed outside the optimizer (init / load): one norm pass; afterwards the
            # update kernel itself produces the next step's norms
            self._norms()
        # (sumsq_next needs no clearing: the step's last launch writes every tensor's sum of its chunk
        # sums, segsum_kernel, in a fixed order)
        self._begun = True

    def _update(self, c0, c1, grad_scale, last):
        """AdamW over chunks [c0, c1); last: then sum the per-chunk norms of ALL tensors (after every
        range of the step has written its chunk sums)."""
        flat = self.flat
        b1, b2 = self.defaults["betas"]
        t = self.step_count
        red = getattr(flat, "grad_reducer", None)
        g16 = red.grad16 if red is not None else None    # all-reduced bf16 gradient buckets
        e0, e1 = c0 * 1024, c1 * 1024
        hyper = (b1, b2, self.defaults["eps"], self.defaults["weight_decay"], float(grad_scale), self.reg_strength,
                 1.0 - b1 ** t, 1.0 - b2 ** t)
        skip = guard_skip(self._guard, c0, c1)
        if c1 > c0:
            K.adamw_step(flat.f32[e0:e1], flat.grad[e0:e1] if g16 is None else None, self.exp_avg[e0:e1],
                         self.exp_avg_sq[e0:e1], flat.chunk_tensor[c0:c1], self.tensor_lr, self.sumsq, flat.bf16[e0:e1],
                         c1 - c0, *hyper, step=self.step_t, sumsq_next=self.sumsq_next, p_f16=flat.f16,
                         f16_range=(flat.f16_lo - e0, flat.f16_hi - e0) if flat.f16 is not None else (0, 0),
                         g_bf16=None if g16 is None else g16[e0:e1], chunk_sq=self.chunk_sq[c0:c1], n_tensors=0,
                         skip=skip)
        if last:   # no update: the fixed-order per-tensor sums over the whole chunk_sq
            K.adamw_step(flat.f32, flat.grad, self.exp_avg, self.exp_avg_sq, flat.chunk_tensor, self.tensor_lr,
                         self.sumsq, None, 0, *hyper, step=self.step_t, sumsq_next=self.sumsq_next,
                         tensor_chunk_off=flat.tensor_chunk_off, chunk_sq=self.chunk_sq)

    def _early_update(self, name):
        rng = self._early.get(name)
        if rng is None or rng in self._done or not self._begun or getattr(self.flat, "grad_reducer", None) is not None:
            return
        self._update(rng[0], rng[1], 1.0, last=False)
        self._done.append(rng)
        self.early_updates += 1

    def update_chunks(self, ranges, grad_scale=1.0):
        """Update the chunk ranges [(c0, c1)] now, ahead of step() (whose remaining update then skips
        them): the data-parallel split step runs this on the collective stream for the buckets whose
        exchange has finished, beside the backward segments still replaying (lrce/graph.py)."""
        self._begin()
        for c0, c1 in ranges:
            if c1 > c0 and (c0, c1) not in self._done:
                self._update(c0, c1, grad_scale, last=False)
                self._done.append((c0, c1))

    def _sync_lrs(self):
        key = tuple(g["lr"] for g in self.param_groups)
        if key == self._lr_cache:
            return
        lrs = torch.zeros(len(self.flat.params))
        for g in self.param_groups:
            for p in g["params"]:
                if p.requires_grad:
                    lrs[self._index[id(p)]] = g["lr"]
        self.tensor_lr.copy_(lrs, non_blocking=True)
        self._lr_cache = key

    @torch.no_grad()
    def step(self, closure=None, grad_scale=1.0):
        loss = closure() if closure is not None else None
        flat = self.flat
        self._begin()
        # the chunk ranges not updated early, in order; the last launch also sums the next norms
        segs, c = [], 0
        for c0, c1 in sorted(self._done):
            if c0 > c:
                segs.append((c, c0))
            c = max(c, c1)
        if c < flat.n_chunks:
            segs.append((c, flat.n_chunks))
        # (early updates ran on the streams that finished those groups' gradients; autograd's
        # end-of-backward join makes this stream wait for them, so their chunk sums are in place)
        for i, (c0, c1) in enumerate(segs):
            self._update(c0, c1, grad_scale, last=i == len(segs) - 1)
        self.sumsq.copy_(self.sumsq_next)
        self._norm_version = flat.master_version()
        flat.mark_bf16_fresh()
        self._begun = False
        self._done = []
        return loss

    def l2_term(self):
        """sum_t ||p_t||_2 of the current parameters (device scalar; no sync)."""
        return self.sumsq.sqrt().sum()

    @torch.no_grad()
    def l2_value(self):
        """The reference's calculate_l2_reg() value (agent_base.py:103-108) for the parameters as they
        are now: the update kernel's norms when they are current, else one multi-tensor norm pass."""
        flat = self.flat
        if self._norm_version != flat.master_version():
            self._norms()
            self._norm_version = flat.master_version()
        return self.l2_term()

    def _norms(self):
        flat = self.flat
        K.l2norm_multi(flat.f32, flat.chunk_tensor, flat.n_chunks, self.sumsq, len(flat.params),
                       tensor_chunk_off=flat.tensor_chunk_off, chunk_sq=self.chunk_sq)

    def zero_grad(self, set_to_none=False, overlap=False):
        """flat.grad = 0 (the backward kernels accumulate into it).  overlap=True: the 1.25 GB clear runs
        on an aux stream beside the forward (which never touches gradients); grad_ready() must then
        be called before the backward (it makes the current stream wait for the clear).  It is issued at
        the step's start, beside the BERT forward (at the recurrent decoder's start instead it measured
        303.2 vs 309.5 QA-samples/s: the decoder's latency chain suffers more from the 1.25 GB stream
        than BERT's)."""
        self.flat.grads_zeroed()
        if not overlap or not self.flat.grad.is_cuda:
            self.flat.grad.zero_()
            return
        dev = self.flat.device
        s = aux_stream(dev, "grad_zero")
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            self.flat.grad.zero_()
        self._zero_stream = s

    def grad_ready(self):
        """Join an overlapped zero_grad (no-op otherwise): call between the forward and the backward."""
        s = getattr(self, "_zero_stream", None)
        if s is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(s)
            self._zero_stream = None

    # ------------------------------------------------------------------ checkpoints
    # torch.optim.AdamW's format: state[i] = {'step', 'exp_avg', 'exp_avg_sq'} per parameter index.
    # The moments are views of the two flat buffers, so torch.save writes each buffer once.
    def state_dict(self):
        flat = self.flat
        step = torch.tensor(float(self._device_step()))
        self.state.clear()
        for p in flat.params:
            if p.requires_grad:
                self.state[p] = {"step": step.clone(), "exp_avg": flat._slice(self.exp_avg, p),
                                 "exp_avg_sq": flat._slice(self.exp_avg_sq, p)}
        try:
            return super().state_dict()
        finally:
            self.state.clear()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        flat = self.flat
        steps = []
        with torch.no_grad():
            for p in flat.params:
                st = self.state.get(p)
                if not st:
                    continue
                flat._slice(self.exp_avg, p).copy_(st["exp_avg"].reshape(p.shape))
                flat._slice(self.exp_avg_sq, p).copy_(st["exp_avg_sq"].reshape(p.shape))
                steps.append(float(st["step"]))
        self.state.clear()
        t = max(steps) if steps else 0.0
        self.step_count = int(t)
        self.step_t.fill_(t)
        self._lr_cache = None
        self._norm_version = None

    def _device_step(self):
        return float(self.step_t.item())

