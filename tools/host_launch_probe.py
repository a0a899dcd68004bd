#!/usr/bin/env python
"""Is the graph-replayed training step host-bound? (dev tool, GPU)  Builds bench.py's model / optimizer /
TrainStepGraph, warms it up, then times N steps twice: host issue time (the loop of step() calls with no
synchronisation) and wall time to the last step's completion, plus the bare hipGraphLaunch host time
of the captured step graph."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vqa-lrce-kbs-2023_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model, opt, reducer, batch = bench.build(10, dev, torch.bfloat16)
    step = bench.make_step(model, opt, reducer, batch, "graph", 1)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{n} steps: host issue {1e3 * (t1 - t0) / n:.2f} ms/step, wall {1e3 * (t2 - t0) / n:.2f} ms/step")
    g = step.__closure__  # the TrainStepGraph object behind the lambda
    tsg = [c.cell_contents for c in g if type(c.cell_contents).__name__ == "TrainStepGraph"][0]
    st = next(iter(tsg.states.values()))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        st.g_step.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"bare replay of the step graph: host {1e3 * (t1 - t0) / n:.2f} ms/launch, wall {1e3 * (t2 - t0) / n:.2f} ms")


if __name__ == "__main__" and not os.environ.get("PROBE_AGENT"):
    main()


def agent_probe():
    """The agent loop (bench.agent_path's setup): host time per next(gen) without synchronisation,
    split into the replay call and the rest."""
    import argparse as _ap
    from lrce.agent import AgentOE
    from lrce.graph import TrainStepGraph
    from lrce.models.e2e import E2EOpenEnded
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    model = E2EOpenEnded(768, 1000, 0.5, (7, 7), 1024, 5, [3], 32, swin_ckpt=None, bert_dir=None)
    a = _ap.Namespace(lr=[5e-6] * 3, reg_strength=0.001, lr_decay_factor=0.5, patience=0.5, min_lr=1e-8,
                      use_cosine_scheduler=False, dataset="msvd-qa-oe", log_dir="/tmp", epoch=1, ckpt_interval=1,
                      debug_mode=True, grad_reduce_dtype="bf16", log_interval=50)
    agent = AgentOE(model, 0, a, log_enabled=False, rank=0)
    batches = [tuple(t.pin_memory() for t in bench.synthetic_batch(10, 2000 + i)) for i in range(4)]
    loader = [batches[i % 4] for i in range(16)]
    spent = {"call": 0.0}
    orig = TrainStepGraph.__call__

    def timed(self, *a, **k):
        t = time.perf_counter()
        r = orig(self, *a, **k)
        spent["call"] += time.perf_counter() - t
        return r
    TrainStepGraph.__call__ = timed
    gen = agent.process_data(loader, True, 0)
    for _ in range(4):
        next(gen)
    torch.cuda.synchronize()
    spent["call"] = 0.0
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        next(gen)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"agent {n} steps: host {1e3 * (t1 - t0) / n:.2f} ms/step (TrainStepGraph call {1e3 * spent['call'] / n:.2f}), "
          f"wall {1e3 * (t2 - t0) / n:.2f} ms/step")


if __name__ == "__main__" and os.environ.get("PROBE_AGENT"):
    agent_probe()
