"""Deterministic per-key weight recipe (TEST INFRASTRUCTURE — oracle side).

Every parameter of the reference state-dict schema (SURVEY.md §8b, 783 keys) is filled from
its own numpy PCG64 stream seeded by (seed, crc32(key)), so the values depend only on the key
name and shape — never on module construction order or on torch's RNG.  The same recipe is
applied to the reference (tests/golden/make_golden.py) and to the MI355X build (tests/), which is
what lets golden fixtures pin the build without shipping 312 M weights.

Scales are chosen so activations stay O(1) through 24 Swin blocks, 12 BERT layers and the
36-step recurrent decoder (non-trivial LN affine params, O(1) attention logits), which makes the
parity tests sensitive to layout/indexing mistakes that near-zero init would hide.
"""
import re
import zlib

import numpy as np
import torch

_LN = re.compile(r"(^|\.)(norm\d*|LayerNorm|layer_norm|fusion_layer_norm)\.(weight|bias)$")


def _scale(key, shape):
    """Return (mean, std) for key."""
    if key.endswith("relative_position_index") or key.endswith("position_ids") or key.endswith("token_type_ids"):
        return None
    m = _LN.search(key)
    if m:
        return (1.0, 0.1) if m.group(3) == "weight" else (0.0, 0.1)
    if key.endswith("relative_position_bias_table"):
        return (0.0, 0.5)
    if "word_embeddings" in key or "position_embeddings" in key or "token_type_embeddings" in key:
        return (0.0, 0.5)
    if ".emb_" in key or key.endswith("summarization_token"):
        return (0.0, 0.3)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return (0.0, 1.0 / np.sqrt(fan_in))
    # 1-D biases
    return (0.0, 0.05)


def value_for(key, shape, seed=0):
    ms = _scale(key, shape)
    if ms is None:
        return None
    mean, std = ms
    rng = np.random.default_rng([seed, zlib.crc32(key.encode())])
    v = rng.standard_normal(tuple(shape), dtype=np.float32) * np.float32(std) + np.float32(mean)
    return torch.from_numpy(v)


def fill_state_dict(template, seed=0):
    """template: mapping key -> tensor (shape/dtype source). Returns a new dict with recipe values
    for parameters; buffers (index tables, position ids) are copied from the template."""
    out = {}
    for k, t in template.items():
        v = value_for(k, t.shape, seed)
        out[k] = t.detach().clone() if v is None else v.to(t.dtype)
    return out


def input_rng(seed):
    return np.random.default_rng([seed, 0x1C3E])


def synthetic_clips(batch, n_scale, seed=1, frames=5, hw=224):
    """(B,S,T,3,H,W) float32 in [0,1) — SURVEY.md §8d."""
    r = input_rng(seed)
    return torch.from_numpy(r.random((batch, n_scale, frames, 3, hw, hw), dtype=np.float32))


def synthetic_question(batch, seq_len, seed=1, q_tokens=20, n_choice=None, ans_tokens=0):
    """BERT-style ids: [CLS]=101, q_tokens-2 ids ~U[1000,30522), [SEP]=102, (answer ids, [SEP]),
    zero padding; attention mask 1 on real tokens; token types 1 on the answer part (MC)."""
    r = np.random.default_rng([seed, 0x7E47])
    shape = (batch,) if n_choice is None else (batch, n_choice)
    ids = np.zeros(shape + (seq_len,), dtype=np.int64)
    mask = np.zeros_like(ids)
    types = np.zeros_like(ids)
    body = q_tokens - 2
    ids[..., 0] = 101
    ids[..., 1:1 + body] = r.integers(1000, 30522, size=shape + (body,))
    ids[..., 1 + body] = 102
    n = q_tokens
    if ans_tokens:
        ids[..., n:n + ans_tokens] = r.integers(1000, 30522, size=shape + (ans_tokens,))
        ids[..., n + ans_tokens] = 102
        types[..., n:n + ans_tokens + 1] = 1
        n = n + ans_tokens + 1
    mask[..., :n] = 1
    return torch.from_numpy(ids), torch.from_numpy(mask), torch.from_numpy(types)
