"""Binding of an nn.Module tree to the native runtime (flat parameter store on one HIP device).

`bind(root)` flattens the root's parameters into a FlatParams and hands the same store to every
submodule (attribute `_lrce_flat`).  Native forward paths call `prepare(module)` which (re)binds on
first use / device change, refreshes the bf16 shadow when masters changed and, when a backward will
follow, makes sure every p.grad is the flat view the kernels accumulate into.
"""

import torch

from .flat import FlatParams


def _set_flat(root, flat):
    for m in root.modules():
        object.__setattr__(m, "_lrce_flat", flat)


def bind(root, device=None):
    params = list(root.parameters())
    if device is None:
        device = params[0].device
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("lrce native modules run on a HIP device only; move the model with .to('cuda')")
    for p in params:
        if p.device != device:
            p.data = p.data.to(device)
    for name, b in root.named_buffers():
        if b.device != device:
            raise RuntimeError(f"buffer {name} not on {device}: call model.to(device) first")
    order = root.lrce_param_order() if hasattr(root, "lrce_param_order") else None
    flat = FlatParams(root, device, order)
    f16 = [p for m in root.modules() if hasattr(m, "lrce_f16_params") for p in m.lrce_f16_params()]
    if f16:
        flat.enable_f16(f16)
    _set_flat(root, flat)
    object.__setattr__(root, "_lrce_root", True)
    return flat


def flat_of(module):
    return getattr(module, "_lrce_flat", None)


def prepare(module):
    """Ensure `module` (any node of a bound tree, or an unbound root) is ready for a native forward."""
    flat = flat_of(module)
    if flat is None or not _valid(module, flat):
        flat = bind(module)
    flat.refresh_bf16()
    if torch.is_grad_enabled() and any(p.requires_grad for p in flat.params):
        flat.attach_grads()
    return flat


def _valid(module, flat):
    """Cheap check that the tree still lives in `flat` (first and last parameter; .to()/.cuda() or
    load_state_dict(assign=True) replace storages and trigger a re-bind)."""
    ps = list(module.parameters())
    for p in (ps[0], ps[-1]):
        if not flat.owns(p) or p.data_ptr() != flat._slice(flat.f32, p).data_ptr():
            return False
    return True


def ensure(module):
    """prepare() at the root of a forward; a bound non-root submodule reuses its tree's store."""
    flat = flat_of(module)
    if flat is not None and not getattr(module, "_lrce_root", False):
        return flat
    return prepare(module)


def needs_grad(*tensors):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


_SIDE_STREAMS = {}
# The stream branches a captured training step may fork into: the set every GPU run of the product has
# captured and replayed.  Two A/B variants that each added one more branch to the captured step crashed
# the HIP runtime in the first captured step (round 4 "fq8", DEBUG_HIP_FORCE_GRAPH_QUEUES=8: graph
# branches on extra queues; round 5 "r5ab2": half of BERT's weight-gradient flush on a sixth stream,
# a new stream whose fork / join pattern nothing else in the step has) — see graph.py and DESIGN §8.
# A new branch is a deliberate change: add its name here after a GPU capture test of it.
AUX_STREAM_NAMES = frozenset({"text", "grad_zero", "decoder_kv", "decoder_wgrad", "swin_bias"})


def _capturing():
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def aux_stream(device, name="text"):
    """A named extra HIP stream of `device`.  "text": the text branch (BERT) runs on it while the
    video branch (Swin) runs on the current stream — the extractors are independent until the fusion
    head, and BERT's small latency-bound launches fill the gaps of Swin's large ones.
    "decoder_wgrad": the recurrent decoder's weight gradients, which feed nothing downstream.
    Refused: a name outside AUX_STREAM_NAMES, and creating a stream while a HIP graph is being captured
    (every stream must exist before the capture: the eager first step creates them)."""
    if name not in AUX_STREAM_NAMES:
        raise ValueError(f"aux stream {name!r} is not one of the captured step's branches "
                         f"{sorted(AUX_STREAM_NAMES)} (runtime.AUX_STREAM_NAMES)")
    key = (torch.device(device).index, name)
    s = _SIDE_STREAMS.get(key)
    if s is None:
        if _capturing():
            raise RuntimeError(f"aux stream {name!r} would be created inside a HIP graph capture: streams "
                               "must exist before the capture (run the step eagerly once first)")
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return s


def join_capture_branches(device):
    """Make the current (capturing) stream wait for every aux stream that is part of the running
    capture: a branch forked into a capture must be joined back before it ends, and a missing join is
    exactly the kind of pattern the runtime answered with a crash instead of an error.  Joining an
    already-joined branch adds an edge and no work.  Returns the number of branches joined."""
    cur = torch.cuda.current_stream(device)
    idx = torch.device(device).index
    n = 0
    for (i, _), st in list(_SIDE_STREAMS.items()):
        if i != idx or st == cur:
            continue
        with torch.cuda.stream(st):
            part = torch.cuda.is_current_stream_capturing()
        if part:
            cur.wait_stream(st)
            n += 1
    return n


def side_stream(device):
    return aux_stream(device, "text")


class _StreamAnchor(torch.autograd.Function):
    """Identity on a one-element leaf token, run on an aux stream: the autograd node inherits that
    stream, so the token's gradient accumulates there and autograd makes the caller's stream wait
    for it at the end of backward (its leaf-stream join) — after everything a backward enqueued on
    the aux stream before this node's turn (it is the earliest node of the forward, hence last)."""

    @staticmethod
    def forward(ctx, token):
        return token.detach().clone()

    @staticmethod
    def backward(ctx, g):
        return g


def stream_anchor(module, stream):
    """A tensor to pass into an autograd Function whose backward forks work onto `stream`; the
    Function returns zeros for it.  None when no backward will run."""
    if not torch.is_grad_enabled():
        return None
    dev = stream.device
    tok = getattr(module, "_lrce_join_token", None)
    if tok is None or tok.device != dev:
        tok = torch.zeros(1, device=dev, requires_grad=True)
        object.__setattr__(module, "_lrce_join_token", tok)
    stream.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(stream):
        return _StreamAnchor.apply(tok)
