"""Generates tests/golden/train_grad_yardstick.json: for every training-parity workload of
tests/test_train_parity_gpu.py (recipe weights seed 0, inputs seed 31, dropout / DropPath off), the
per-tensor gradient error of the CPU oracle run under the reference's own mixed precision and under
bf16, both against the same oracle in fp32 (max|d| / max|ref| per tensor; for the analytically-zero
BERT key biases, max|grad| / max|fp32 query-bias grad|).

The reference trains under torch.cuda.amp.autocast (fp16) with a GradScaler (agent_oe.py:28,40-42,
agent_base.py:45).  CPU autocast is NOT that policy (on the CPU it runs layer_norm and softmax in the
low-precision dtype, which CUDA autocast keeps in f32), so the oracle runs under `CudaAutocast`
instead, a TorchFunctionMode restating the CUDA policy for the ops the oracle uses: F.linear,
F.conv3d and matmul take operands rounded to the low-precision dtype, accumulate in f32 and round
their output (and, through the casts' autograd, the gradients flowing through them), everything else
— LayerNorm, softmax, GELU, residual adds, the losses — runs in f32.  fp16 runs with a GradScaler
restatement: loss x 2^16, halved until every gradient is finite, gradients divided back.

The parity test reads this only to PRINT how its own error compares with the reference's numerics
on each tensor (the bars themselves are fixed constants).

Run in a container with the repo (not the reference): python tests/golden/make_train_yardstick.py
(about 10 min on 8 cores)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "vqa-lrce-kbs-2023_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.overrides import TorchFunctionMode  # noqa: E402

from helpers import oracle_sd, rel  # noqa: E402
from oracle import lrce_oracle as O  # noqa: E402


class CudaAutocast(TorchFunctionMode):
    """torch.cuda.amp.autocast's policy for the oracle's ops (see the module docstring)."""
    GEMM = {F.linear, F.conv3d, torch.matmul, torch.Tensor.__matmul__, torch.Tensor.matmul}

    def __init__(self, dtype):
        super().__init__()
        self.dtype = dtype

    def _round(self, t):
        if isinstance(t, torch.Tensor) and t.is_floating_point():
            return t.to(self.dtype).to(torch.float32)
        return t

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in self.GEMM:
            out = func(*[self._round(a) for a in args], **{k: self._round(v) for k, v in kwargs.items()})
            return self._round(out)
        return func(*args, **kwargs)


def grads(filled, inputs, task, dtype):
    import test_train_parity_gpu as T
    clips, ids, mask, types, label = inputs
    scale = 65536.0 if dtype == torch.float16 else 1.0
    while True:
        sd = oracle_sd(filled, requires_grad=True)
        if dtype is None:
            y = O.e2e_forward(sd, clips, ids, mask, types, task)
        else:
            with CudaAutocast(dtype):
                y = O.e2e_forward(sd, clips, ids, mask, types, task)
        (T.oracle_loss(task, y, label) * scale).backward()
        g = {k: v.grad / scale for k, v in sd.items() if v.is_floating_point() and v.grad is not None}
        if all(bool(torch.isfinite(t).all()) for t in g.values()):
            return g, y.detach()
        scale /= 2  # GradScaler: skip the step, halve the scale


def main():
    import test_train_parity_gpu as T
    torch.set_num_threads(os.cpu_count() or 8)
    out = {}
    for name, batch in T.WORKLOADS:
        filled, task, L = T.recipe(name)
        inputs = T._inputs(name, batch, seed=T.SEED)
        g32, y = grads(filled, inputs, task, None)
        if task == "count":
            print(name, "positive outputs:", int((y > 0).sum()), "of", batch, flush=True)
        ent = {}
        for tag, dt in (("fp16", torch.float16), ("bf16", torch.bfloat16)):
            g, _ = grads(filled, inputs, task, dt)
            for k, ref in g32.items():
                if k.endswith("attention.self.key.bias"):
                    # analytically zero: record max|key-bias grad| / max|fp32 query-bias grad| instead
                    qb = g32[k.replace("key.bias", "query.bias")]
                    ent.setdefault(k, {})[tag] = round(float(g[k].abs().max() / qb.abs().max()), 6)
                elif float(ref.abs().max()) > 0:
                    ent.setdefault(k, {})[tag] = round(rel(g[k], ref), 6)
        out[f"{name}_b{batch}"] = ent
        worst = max(ent.items(), key=lambda kv: kv[1].get("fp16", 0))
        print(name, batch, len(ent), "worst fp16:", worst, flush=True)
    with open(os.path.join(HERE, "train_grad_yardstick.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
