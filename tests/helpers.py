"""Shared test helpers: load the deterministic weight recipe into product modules, relative errors."""
import torch

from oracle import weights as W


def load_recipe(module, prefix="", seed=0):
    """Fill `module` (product nn.Module) with recipe values for keys prefix+name; returns the f32 CPU
    state dict (with prefix) for the oracle."""
    tmpl = {prefix + k: v for k, v in module.state_dict().items()}
    filled = W.fill_state_dict({k: v.cpu() for k, v in tmpl.items()}, seed)
    module.load_state_dict({k[len(prefix):]: v for k, v in filled.items()}, strict=True)
    return filled


def rel(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def oracle_sd(filled, requires_grad=False):
    out = {}
    for k, v in filled.items():
        t = v.detach().clone().float() if v.is_floating_point() else v.clone()
        if requires_grad and t.is_floating_point():
            t.requires_grad_(True)
        out[k] = t
    return out
