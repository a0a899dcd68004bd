"""bench.py's rank launcher (reference: train_ddp.py:136-138 spawns world_size = device_count
processes).  `python bench.py --gpus N` started plainly must launch N ranks itself (children through
torch.distributed.run, before any GPU call) and report the joined world; a world that differs from
--gpus is an error.  Checked in --dry-run mode: gloo ranks on the CPU, no model, no GPU."""
import json
import os
import subprocess
import sys

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH] + args, env=env, cwd="/tmp", capture_output=True, text=True,
                       timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


def test_launcher_spawns_n_ranks():
    rc, lines, err = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1"])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, (lines, err[-2000:])      # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["grad_reduce"] == "bf16"


def test_single_gpu_needs_no_launcher():
    rc, lines, err = _run(["--gpus", "1", "--dry-run"])
    assert rc == 0, err[-2000:]
    assert json.loads(lines[0])["n_gpus"] == 1


def test_world_mismatch_is_an_error():
    # started as one rank of a 1-process world (WORLD_SIZE set: no launch) but asked for 2 GPUs
    rc, lines, err = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and not lines
    assert "--gpus 2" in err


def test_dev_only_work_skipping_variables_are_refused():
    # a stray LRCE_DEV_* export must never yield a (silently inflated) headline
    rc, lines, err = _run(["--gpus", "1", "--dry-run"], {"LRCE_DEV_SWIN_S3": "9"})
    assert rc != 0 and not lines
    assert "LRCE_DEV_SWIN_S3" in err


def test_non_default_switches_are_recorded():
    rc, lines, err = _run(["--gpus", "1", "--dry-run"], {"LRCE_DEC_FUSED": "blocks"})
    assert rc == 0, err[-2000:]
    assert json.loads(lines[0])["lrce_env"] == {"LRCE_DEC_FUSED": "blocks"}


def test_product_reads_no_dev_only_variables():
    # the work-skipping sensitivity knobs are gone from the product sources (their A/Bs are recorded
    # in DESIGN.md / profiles/r5_bench_sensitivity_ab.txt)
    pkg = os.path.join(REPO, "vqa-lrce-kbs-2023_amd")
    hits = []
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                with open(os.path.join(root, f)) as fh:
                    if "LRCE_DEV_" in fh.read():
                        hits.append(f)
    assert not hits, hits
