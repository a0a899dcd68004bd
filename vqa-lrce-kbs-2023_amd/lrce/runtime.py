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


def aux_stream(device, name="text"):
    """A named extra HIP stream of `device`.  "text": the text branch (BERT) runs on it while the
    video branch (Swin) runs on the current stream — the extractors are independent until the fusion
    head, and BERT's small latency-bound launches fill the gaps of Swin's large ones.
    "decoder_wgrad": the recurrent decoder's weight gradients, which feed nothing downstream."""
    key = (torch.device(device).index, name)
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return s


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
