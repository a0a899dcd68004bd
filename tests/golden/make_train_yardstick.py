"""Generates tests/golden/train_grad_yardstick.json: for the two training-parity workloads of
tests/test_train_parity_gpu.py (msvd-qa-oe bs 10 CE, tgif-transition MC bs 9 hinge; recipe weights
seed 0, inputs seed 31, dropout / DropPath off), the per-tensor gradient error of the CPU oracle run
under the reference's own mixed precision — torch.autocast fp16, as agent_oe.py:28 /
agent_mc.py:52 train — and under bf16 autocast, both against the same oracle in fp32
(max|d| / max|ref| per tensor; for the analytically-zero BERT key biases, max|grad| / max|fp32
query-bias grad|).  The parity test allows a tensor its family bar, or the reference's own fp16
training error, or half its bf16 error, whichever is largest: the HIP path must be at least as close
to fp32 as the reference's own mixed-precision numerics are.

Run in a container with the repo (not the reference): python tests/golden/make_train_yardstick.py
(about 1.5 min per workload on 8 cores)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "vqa-lrce-kbs-2023_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from helpers import oracle_sd, rel  # noqa: E402
from oracle import lrce_oracle as O  # noqa: E402
from oracle import weights as W  # noqa: E402


def grads(filled, inputs, task, dtype):
    clips, ids, mask, types, label = inputs
    sd = oracle_sd(filled, requires_grad=True)
    with torch.autocast("cpu", dtype=dtype or torch.bfloat16, enabled=dtype is not None):
        y = O.e2e_forward(sd, clips, ids, mask, types, task)
    y = y.float()
    loss = O.hinge_loss(y, label, 1.0) if task == "mc" else F.cross_entropy(y, label, ignore_index=-100)
    loss.backward()
    return {k: v.grad for k, v in sd.items() if v.is_floating_point() and v.grad is not None}


def main():
    import test_train_parity_gpu as T
    from lrce.models import e2e
    out = {}
    for name, batch in T.WORKLOADS:
        task, ncls, L = T.CFG[name]
        cls = {"oe": e2e.E2EOpenEnded, "mc": e2e.E2EMultipleChoice}[task]
        m = cls(768, ncls, 0.0, (7, 7), 1024, 5, [3], L)
        filled = W.fill_state_dict({k: v for k, v in m.state_dict().items()}, 0)
        del m
        inputs = T._inputs(task, batch, L, seed=T.SEED)
        g32 = grads(filled, inputs, task, None)
        ent = {}
        for tag, dt in (("fp16", torch.float16), ("bf16", torch.bfloat16)):
            g = grads(filled, inputs, task, dt)
            for k, ref in g32.items():
                if k.endswith("attention.self.key.bias"):
                    # analytically zero: record max|key-bias grad| / max|fp32 query-bias grad| instead
                    qb = g32[k.replace("key.bias", "query.bias")]
                    ent.setdefault(k, {})[tag] = round(float(g[k].abs().max() / qb.abs().max()), 6)
                elif float(ref.abs().max()) > 0:
                    ent.setdefault(k, {})[tag] = round(rel(g[k], ref), 6)
        out[f"{name}_b{batch}"] = ent
        print(name, batch, len(ent), flush=True)
    with open(os.path.join(HERE, "train_grad_yardstick.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
