"""bench.py's own N = 2 model path on the one-GPU box (reference: train_ddp.py:10-13,136-138 — one
process per GPU, DDP gradient all-reduce).  The driver's scaling run executes `bench.py --gpus N` over
RCCL on an 8-GPU node; this test runs the same code on one GPU with --shared-device: both ranks on
cuda:0, exchanging over gloo, with everything else as the N-GPU run uses it — the launcher, the split
backward at SPLIT_SWIN_STAGE, bf16 gradient buckets, the graph-replayed step with the early-update
graphs behind each bucket exchange, max-over-ranks timing.  Asserts the JSON line's world and
parallelism, a finite loss, and bit-identical replicas after the steps (replica_digest over every f32
master weight).  The children's log goes to gpurun_out/bench_dp2_rehearsal.log."""
import json
import math
import os
import subprocess
import sys

import pytest

from conftest import REPO, gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


@pytest.mark.timeout(600)
def test_bench_two_rank_model_path_on_one_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    log = os.path.join(REPO, "gpurun_out", "bench_dp2_rehearsal.log")
    with open(log, "w") as err:
        p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--shared-device",
                            "--steps", "2", "--warmup", "2", "--no-cpu-baseline", "--agent-steps", "0",
                            "--roofline-steps", "1"], env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=err,
                           text=True, timeout=560)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    tail = open(log).read()[-3000:]
    assert p.returncode == 0, tail
    assert len(lines) == 1, (p.stdout[-2000:], tail)
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["grad_reduce"] == "bf16"
    assert out["config"]["split_swin_stage"] is not None
    assert out["config"]["global_batch"] == 20
    assert math.isfinite(out["loss"]) and out["value"] > 0
    assert out["replicas_identical"] is True
    assert "rehearsal" in out
