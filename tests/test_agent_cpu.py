"""CPU tests of the agent / CLI layer (reference args.py, parser.py, lrce/agent/*): argument surface and
post-processing, losses vs the reference's own loop formulation, learning-rate schedules, and the
synthetic dataset's item contract (e2e_dataset.py:118-124).  No GPU and no native compute here."""
import math

import pytest
import torch

from lrce import cli
from lrce.agent.agent_mc import hinge_loss
from lrce.agent.schedulers import CosineAnnealingWarmupRestarts, ReduceLROnPlateau
from lrce.dataset import SyntheticQADataset


# ------------------------------------------------------------------------------------------ CLI
def test_train_ddp_defaults_and_config_merge():
    a = cli.parse_arg_train(["--dataset", "msvd-qa-oe", "--synthetic", "8"])
    assert a.temporal_scale == [3] and a.batch_size == 20 and a.epoch == 20 and a.drop_out_rate == 0.5
    assert a.lr == [5e-6] * 3 and a.reg_strength == 0.001 and a.min_lr == 1e-8
    assert (a.feature_dim, a.text_seq_len, a.num_classes, a.task_type) == (768, 32, 1000, "oe")
    assert a.video_feature_res == [7, 7] and a.video_feature_dim == 1024 and a.frame_sample_size == 5
    # plateau scheduler: the cosine-only flags are deleted (parser.py:96-101); no hinge -> no margin
    for gone in ("lr_restart_epoch", "lr_restart_mul", "lr_warm_up", "margin", "comment"):
        assert not hasattr(a, gone)
    assert a.patience == 0.5


def test_train_args_py_defaults_and_cosine_branch():
    a = cli.parse_arg_train(["--dataset", "tgif-transition", "--synthetic", "8", "--use-cosine-scheduler",
                             "--use-hinge-loss", "--lr", "1e-4", "2e-5", "3e-6", "--comment", "x"],
                            temporal_default=(1, 2, 3))
    assert a.temporal_scale == [1, 2, 3] and a.lr == [1e-4, 2e-5, 3e-6]
    assert not hasattr(a, "patience") and a.lr_restart_epoch == 2 and a.lr_warm_up == 0.1
    assert a.margin == 1.0 and a.comment == "x" and a.task_type == "mc" and a.text_seq_len == 40


def test_msrvtt_config_overrides_dataset_string():
    """configs/msrvtt-qa-oe.json carries "msvrvtt-qa-oe"; the reference's merge copies it into args."""
    a = cli.parse_arg_train(["--dataset", "msrvtt-qa-oe", "--synthetic", "8"])
    assert a.dataset == "msvrvtt-qa-oe" and a.num_classes == 1500 and a.text_seq_len == 37


def test_eval_parser():
    a = cli.parse_arg_eval(["--dataset", "tgif-count", "--model-path", "x.pt", "--synthetic", "4"])
    assert a.reg_strength == 0 and a.temporal_scale == [3] and a.task_type == "count" and a.batch_size == 20
    with pytest.raises(SystemExit):
        cli.parse_arg_eval(["--dataset", "tgif-count", "--synthetic", "4"])          # --model-path required
    with pytest.raises(SystemExit):
        cli.parse_arg_train(["--dataset", "msvd-qa-oe"])                               # no data source
    with pytest.raises(SystemExit):
        cli.parse_arg_train(["--dataset", "ucf101", "--synthetic", "4"])               # not a reference choice


def test_factories():
    from lrce.agent import AgentCount, AgentMC, AgentOE
    from lrce.models.e2e import E2ECount, E2EMultipleChoice, E2EOpenEnded
    assert cli.factories("oe") == (E2EOpenEnded, AgentOE)
    assert cli.factories("mc") == (E2EMultipleChoice, AgentMC)
    assert cli.factories("count") == (E2ECount, AgentCount)
    with pytest.raises(SystemExit):
        cli.factories("ranking")


# ------------------------------------------------------------------------------------------ losses
def _ref_hinge(out, gt, margin):
    """agent_mc.py:20-41, tensor-for-tensor (per-sample loop, concat without the correct index)."""
    batch, total_mc = out.shape
    losses = []
    for i in range(batch):
        c = int(gt[i])
        correct = out[i][c]
        total = torch.zeros(total_mc)
        for j in range(total_mc):
            if j != c:
                total[j] = out[i][j] - correct
        total = torch.cat((total[:c], total[c + 1:])) + margin
        total = torch.max(total, torch.zeros(total_mc - 1))
        losses.append(total.sum())
    return torch.stack(losses).mean()


@pytest.mark.parametrize("margin", [1.0, 0.2])
def test_hinge_loss_value_and_grad_match_reference_loop(margin):
    g = torch.Generator().manual_seed(3)
    out = (torch.randn(9, 5, generator=g) * 2).requires_grad_(True)
    gt = torch.randint(0, 5, (9,), generator=g)
    out2 = out.detach().clone().requires_grad_(True)
    ref = _ref_hinge(out2, gt, margin)
    ours = hinge_loss(out, gt, margin)
    assert abs(float(ours) - float(ref)) < 1e-6
    ours.backward()
    ref.backward()
    assert torch.allclose(out.grad, out2.grad, atol=1e-7)


# ------------------------------------------------------------------------------------------ schedules
def _opt(n_groups=3, lr=1e-3):
    ps = [torch.nn.Parameter(torch.zeros(2)) for _ in range(n_groups)]
    return torch.optim.AdamW([{"params": [p], "lr": lr} for p in ps], lr=lr)


def test_cosine_warmup_restarts_shape():
    opt = _opt()
    s = CosineAnnealingWarmupRestarts(opt, first_cycle_steps=10, cycle_mult=1.0, max_lr=1e-3, min_lr=1e-5,
                                      warmup_steps=2, gamma=0.5)
    lrs = [opt.param_groups[0]["lr"]]
    for _ in range(25):
        s.step()
        lrs.append(opt.param_groups[0]["lr"])
    assert lrs[0] == pytest.approx(1e-5)                       # starts at min_lr
    assert lrs[1] == pytest.approx(1e-5 + (1e-3 - 1e-5) / 2)   # linear warm-up
    assert lrs[2] == pytest.approx(1e-3)                       # peak at the end of warm-up
    mid = 1e-5 + (1e-3 - 1e-5) * (1 + math.cos(math.pi * 4 / 8)) / 2
    assert lrs[6] == pytest.approx(mid)                        # half-cosine over the rest of the cycle
    assert lrs[10] == pytest.approx(1e-5)                      # restart: back to min_lr ...
    assert lrs[12] == pytest.approx(5e-4)                      # ... peaks at max_lr * gamma
    assert all(g["lr"] == lrs[-1] for g in opt.param_groups)


def test_cosine_fractional_epochs_as_reference_steps_it():
    """agent_base.py:138 steps with epoch + i / len(dl) and warmup_steps = 0.1 (a fraction of an epoch)."""
    opt = _opt()
    s = CosineAnnealingWarmupRestarts(opt, first_cycle_steps=2, cycle_mult=1, max_lr=5e-6, min_lr=1e-8,
                                      warmup_steps=0.1, gamma=0.5)
    s.step(0.05)
    assert opt.param_groups[0]["lr"] == pytest.approx(1e-8 + (5e-6 - 1e-8) * 0.5)
    s.step(0.1)
    assert opt.param_groups[0]["lr"] == pytest.approx(5e-6)
    s.step(2.1)     # second cycle (epoch 2 = first_cycle_steps): peak halves
    assert s.cycle == 1 and opt.param_groups[0]["lr"] == pytest.approx(2.5e-6)


def test_plateau_scheduler_accepts_reference_defaults():
    opt = _opt(lr=5e-6)
    s = ReduceLROnPlateau(opt, mode="max", factor=0.5, patience=0.5, min_lr=1e-8)
    s.step(0.5)
    s.step(0.4)      # worse than best for > patience epochs -> decay
    assert opt.param_groups[0]["lr"] == pytest.approx(2.5e-6)


# ------------------------------------------------------------------------------------------ data
@pytest.mark.parametrize("task,L,ts", [("oe", 32, [3]), ("mc", 40, [1, 2, 3]), ("count", 30, [3])])
def test_synthetic_item_contract(task, L, ts):
    d = SyntheticQADataset(6, task, L, ts, num_classes=1000, seed=1)
    clips, ids, mask, types, gt = d[2]
    S = sum(ts)
    assert clips.shape == (S, 5, 3, 224, 224) and clips.dtype == torch.float32
    assert 0.0 <= float(clips.min()) and float(clips.max()) < 1.0
    shp = (5, L) if task == "mc" else (L,)
    assert ids.shape == shp and mask.shape == shp and types.shape == shp and ids.dtype == torch.int64
    row = ids[0] if task == "mc" else ids
    assert int(row[0]) == 101 and int(row[19]) == 102 and int(mask.reshape(-1, L)[0].sum()) == (25 if task == "mc" else 20)
    if task == "mc":
        assert int(types[0].sum()) == 5 and 0 <= int(gt) < 5 and gt.dtype == torch.int64
    elif task == "count":
        assert gt.dtype == torch.float32 and gt.dim() == 0
    else:
        assert 0 <= int(gt) < 1000 and gt.dtype == torch.int64
    again = d[2]
    assert all(torch.equal(a, b) for a, b in zip((clips, ids, mask, types, gt), again))


def test_synthetic_loader_and_distributed_split():
    from torch.utils.data.distributed import DistributedSampler
    d = SyntheticQADataset(10, "oe", 32, [1], seed=0)
    idx = [list(DistributedSampler(d, num_replicas=2, rank=r, shuffle=False)) for r in range(2)]
    assert sorted(idx[0] + idx[1]) == list(range(10)) and not set(idx[0]) & set(idx[1])
    dl = torch.utils.data.DataLoader(d, batch_size=4, sampler=DistributedSampler(d, 2, 0, shuffle=False))
    b = next(iter(dl))
    assert b[0].shape == (4, 1, 5, 3, 224, 224) and b[1].shape == (4, 32) and b[4].shape == (4,)


def test_datasets_builder_requires_synthetic():
    a = cli.parse_arg_train(["--dataset", "msvd-qa-oe", "--dataset-dir", "/nonexistent"])
    with pytest.raises(NotImplementedError):
        cli.datasets(a, ["train"])
    a = cli.parse_arg_train(["--dataset", "tgif-transition", "--synthetic", "12", "--batch-size", "2"])
    tr, va = cli.datasets(a, ["train", "test"])
    assert len(tr) == 12 and len(va) == 3 and tr[0][1].shape == (5, 40)


class _StubOE(torch.nn.Module):
    """Stands in for the native E2E model in the CPU plumbing test (the product model runs on the GPU
    only): deterministic logits from the inputs."""

    def __init__(self, ncls):
        super().__init__()
        self.w = torch.nn.Parameter(torch.linspace(-1, 1, ncls))


    def forward(self, clips, ids, mask, types):
        key = clips.mean(dim=(1, 2, 3, 4, 5)) * 1000 + ids.float().sum(1)
        return torch.outer(key, self.w)


def test_config1_cpu_eval_plumbing(monkeypatch):
    """BASELINE config 1 (msvd-qa-oe, batch 2, temporal scale 3, eval on 4 synthetic clips): the
    eval.py plumbing — parser -> dataset -> loader -> agent.process_data -> metric reduction — on
    the CPU with a stub model.  The product model itself has no CPU path by design."""
    import lrce.agent.agent_base as AB
    from lrce.agent import AgentOE
    monkeypatch.setattr(AB, "ensure", lambda m: None)      # the stub has no native flat store
    a = cli.parse_arg_eval(["--dataset", "msvd-qa-oe", "--model-path", "unused.pt", "--batch-size", "2",
                            "--temporal-scale", "3", "--synthetic", "4", "--num-workers", "0"])
    (test_ds,) = cli.datasets(a, ["test"])
    assert len(test_ds) == 4
    dl = torch.utils.data.DataLoader(test_ds, batch_size=a.batch_size, shuffle=False)
    model = _StubOE(a.num_classes)
    agent = AgentOE(model, "cpu", a, False, True)
    agent.do_evaluation(dl)
    correct, total, losses = 0, 0, []
    with torch.no_grad():
        for clips, ids, mask, types, gt in dl:
            out = model(clips, ids, mask, types)
            correct += int((out.argmax(1) == gt).sum())
            total += gt.numel()
            losses.append(float(torch.nn.functional.cross_entropy(out, gt)))
    assert agent.last_metric_val == pytest.approx(correct / total)
    nz = [x for x in losses if x != 0]
    assert agent.last_loss == pytest.approx(sum(nz) / len(nz), rel=1e-5)


def test_graph_capture_refuses_the_crashing_hip_debug_queue_knob(monkeypatch):
    """DEBUG_HIP_FORCE_GRAPH_QUEUES=8 crashed the HIP runtime at the first captured step (round-4
    A/B "fq8", reproduced in round 5): the capture refuses it with an explanation."""
    from lrce import graph
    monkeypatch.setenv("DEBUG_HIP_FORCE_GRAPH_QUEUES", "8")
    with pytest.raises(RuntimeError, match="DEBUG_HIP_FORCE_GRAPH_QUEUES"):
        graph._check_runtime_env()
    monkeypatch.setenv("DEBUG_HIP_FORCE_GRAPH_QUEUES", "0")
    graph._check_runtime_env()


def test_graph_capture_refuses_unregistered_or_in_capture_streams(monkeypatch):
    """The round-5 capture-time SIGSEGV ("r5ab2": half of BERT's weight-gradient flush on a new sixth
    stream) and the round-4 one share one trait: one more stream branch in the captured step.  The
    runtime refuses a branch name outside the captured-and-replayed set, and creating a stream while a
    graph is being captured; graph.py joins every branch forked into a capture (join_capture_branches)."""
    from lrce import runtime as R
    with pytest.raises(ValueError, match="AUX_STREAM_NAMES"):
        R.aux_stream(torch.device("cuda", 0), "text_flush2")
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    monkeypatch.setattr(R, "_SIDE_STREAMS", {})
    with pytest.raises(RuntimeError, match="inside a HIP graph capture"):
        R.aux_stream(torch.device("cuda", 0), "decoder_wgrad")
    for name in ("text", "grad_zero", "decoder_kv", "decoder_wgrad", "swin_bias"):
        assert name in R.AUX_STREAM_NAMES
    from lrce import graph
    assert graph.join_capture_branches is R.join_capture_branches
