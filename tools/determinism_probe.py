#!/usr/bin/env python
"""Which fusion-head gradients are not bit-reproducible run to run (dev probe, GPU): the OE head
forward + backward twice per setting of fusionv3._KV_ASYNC / _WGRAD_EARLY, same seeds; prints the
tensors whose two runs differ and the largest relative difference."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

from lrce.models import fusionv3 as F  # noqa: E402


def run(m, vf, tf):
    m.zero_grad(set_to_none=True)
    vg, tg = vf.clone().requires_grad_(True), tf.clone().requires_grad_(True)
    torch.manual_seed(11)
    y = m(vg, tg, None)
    R = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).cuda()
    (y.float() * R).sum().backward()
    torch.cuda.synchronize()
    out = {"y": y.detach().float().clone(), "dv": vg.grad.clone(), "dt": tg.grad.clone()}
    out.update({k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None})
    return out


_BWD = F._RecurrentDecoderFn.backward


def _spy(ctx, ds):
    out = _BWD(ctx, ds)
    _spy.seen.append(out[0].detach().clone())   # d(video memory) of the decoder
    return out


_spy.seen = []


def diff(a, b):
    bad = []
    for k in a:
        if not torch.equal(a[k], b[k]):
            d = (a[k] - b[k]).abs().max().item() / max(a[k].abs().max().item(), 1e-30)
            bad.append(f"{k} ({d:.1e})")
    return bad


def main():
    torch.manual_seed(3)
    m = F.LRCEOpenEnded(768, 1000, 0.1, (7, 7), 1024, 5, [3], 32).cuda().train()
    vf = torch.randn(3, 3, 3, 49, 1024, device="cuda")
    tf = torch.randn(3, 32, 768, device="cuda")
    F._RecurrentDecoderFn.backward = staticmethod(_spy)
    res = {}
    for kv, early in ((False, False), (True, False), (False, True), (True, True)):
        F._KV_ASYNC, F._WGRAD_EARLY = kv, early
        a, b = run(m, vf, tf), run(m, vf, tf)
        a["decoder_dv"], b["decoder_dv"] = _spy.seen[-2], _spy.seen[-1]
        res[(kv, early)] = a
        bad = diff(a, b)
        print(f"kv_async={kv} wgrad_early={early}: {len(bad)} of {len(a)} differ run to run: {bad[:8]}", flush=True)
    for x, y in (((False, False), (True, False)), ((False, False), (False, True))):
        bad = diff(res[x], res[y])
        print(f"{x} vs {y}: {len(bad)} differ: {bad[:12]}", flush=True)


if __name__ == "__main__":
    main()
