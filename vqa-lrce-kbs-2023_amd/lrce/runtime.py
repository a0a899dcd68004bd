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


def side_stream(device):
    """The second HIP stream of `device` that the text branch (BERT) runs on while the video branch
    (Swin) runs on the current stream: the two extractors are independent until the fusion head, and
    BERT's small latency-bound launches fill the gaps of Swin's large ones."""
    key = torch.device(device).index
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return s
