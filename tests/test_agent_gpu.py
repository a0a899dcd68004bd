"""GPU tests of the agent / CLI layer on the native path (reference lrce/agent/*.py, train_ddp.py,
eval.py): the reported loss is the reference's task loss + reg * sum ||p||_2, a train step updates the
weights, hinge / MSE heads, checkpoint round trip in the `{'model_state_dict'}` format, and the
train_ddp.py -> eval.py scripts end to end on synthetic data (one rank, RCCL process group)."""
import argparse
import glob
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

from conftest import PKG, gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _args(tmp_path, **kw):
    a = dict(lr=[1e-4] * 3, reg_strength=0.001, lr_decay_factor=0.5, patience=0.5, min_lr=1e-8,
             use_cosine_scheduler=False, dataset="msvd-qa-oe", log_dir=str(tmp_path), epoch=1, ckpt_interval=1,
             use_hinge_loss=False, margin=1.0, debug_mode=True)
    a.update(kw)
    return argparse.Namespace(**a)


def _batch(task, L, n=2, ncls=50):
    from lrce.dataset import SyntheticQADataset
    d = SyntheticQADataset(n, task, L, [1], num_classes=ncls, seed=5)
    items = [d[i] for i in range(n)]
    return [torch.stack([it[k] for it in items]) for k in range(5)]


def _l2(model):
    return sum(p.detach().double().norm(2) for p in model.parameters() if p.requires_grad).item()


def _model(task, ncls, L):
    from lrce.models.e2e import E2ECount, E2EMultipleChoice, E2EOpenEnded
    cls = {"oe": E2EOpenEnded, "mc": E2EMultipleChoice, "count": E2ECount}[task]
    torch.manual_seed(0)
    return cls(768, ncls, 0.5, (7, 7), 1024, 5, [1], L)


def test_agent_oe_loss_and_update(tmp_path):
    from lrce.agent import AgentOE
    agent = AgentOE(_model("oe", 50, 32), 0, _args(tmp_path), log_enabled=False)
    b = _batch("oe", 32)
    with torch.no_grad():
        agent.model.eval()
        out = agent.model(*(t.cuda() for t in b[:4])).float()
        loss, correct, total = agent.step(*b, is_train=False)
    expect = F.cross_entropy(out, b[4].cuda()).item() + 0.001 * _l2(agent.model.module)
    assert abs(loss - expect) < 1e-3 * abs(expect), (loss, expect)
    assert total == 2 and 0 <= correct <= 2
    w0 = agent.model.module.fusion_model.final_fc.weight.detach().clone()
    agent.model.train()
    loss_t, _, _ = agent.step(*b, is_train=True)
    torch.cuda.synchronize()
    assert loss_t == loss_t and not torch.equal(w0, agent.model.module.fusion_model.final_fc.weight.detach())
    # the L2 value after the update comes from the optimizer kernel's norms: must equal a fresh count
    assert abs(agent.calculate_l2_reg().item() - _l2(agent.model.module)) < 1e-4 * _l2(agent.model.module)


def test_agent_mc_hinge_and_count_mse(tmp_path):
    from lrce.agent import AgentCount, AgentMC
    from lrce.agent.agent_mc import hinge_loss
    agent = AgentMC(_model("mc", 1, 40), 0, _args(tmp_path, use_hinge_loss=True, margin=1.0), log_enabled=False)
    b = _batch("mc", 40)
    with torch.no_grad():
        agent.model.eval()
        out = agent.model(*(t.cuda() for t in b[:4])).float()
        loss, correct, total = agent.step(*b, is_train=False)
    assert out.shape == (2, 5)
    expect = hinge_loss(out, b[4].cuda(), 1.0).item() + 0.001 * _l2(agent.model.module)
    assert abs(loss - expect) < 1e-3 * abs(expect)
    loss_t, _, _ = agent.step(*b, is_train=True)
    assert loss_t == loss_t
    del agent
    agent = AgentCount(_model("count", 1, 30), 0, _args(tmp_path, dataset="tgif-count"), log_enabled=False)
    b = _batch("count", 30)
    with torch.no_grad():
        agent.model.eval()
        out = agent.model(*(t.cuda() for t in b[:4])).float()
        loss, mse = agent.step(*b, is_train=False)
    assert mse.shape == (2,)
    assert torch.allclose(mse, (out - b[4].cuda()) ** 2, rtol=1e-5)
    loss_t, mse_t = agent.step(*b, is_train=True)
    assert loss_t == loss_t and mse_t.shape == (2,)


def test_checkpoint_round_trip(tmp_path):
    from lrce.agent import AgentOE
    a = _args(tmp_path)
    a.ckpt_dir = str(tmp_path)
    agent = AgentOE(_model("oe", 50, 32), 0, a, log_enabled=False)
    b = _batch("oe", 32)
    agent.model.train()
    agent.step(*b, is_train=True)
    path = agent.save_checkpoint(1, "best")
    assert set(torch.load(path, weights_only=True)) == {"model_state_dict"}
    agent.model.eval()
    with torch.no_grad():
        y0 = agent.model(*(t.cuda() for t in b[:4])).float()
    fresh = AgentOE(_model("oe", 50, 32), 0, _args(tmp_path, reg_strength=0.0), log_enabled=False, is_eval=True)
    fresh.load_checkpoint(path)
    fresh.model.eval()
    with torch.no_grad():
        y1 = fresh.model(*(t.cuda() for t in b[:4])).float()
    assert torch.allclose(y0, y1, atol=1e-5, rtol=1e-5)


def test_train_ddp_then_eval_scripts(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29517", HIP_VISIBLE_DEVICES="0")
    common = ["--temporal-scale", "1", "--batch-size", "2", "--num-workers", "0"]
    r = subprocess.run([sys.executable, os.path.join(PKG, "train_ddp.py"), "--dataset", "msvd-qa-oe", "--synthetic", "4",
                        "--synthetic-val", "2", "--epoch", "1", "--log-dir", str(tmp_path), "--lr", "1e-4"] + common,
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    ckpts = glob.glob(os.path.join(str(tmp_path), "*_msvd-qa-oe", "weights", "*.pt"))
    assert any(c.endswith("best.pt") for c in ckpts) and len(ckpts) == 2, ckpts
    assert os.path.exists(glob.glob(os.path.join(str(tmp_path), "*_msvd-qa-oe", "config.json"))[0])
    best = [c for c in ckpts if c.endswith("best.pt")][0]
    r = subprocess.run([sys.executable, os.path.join(PKG, "eval.py"), "--dataset", "msvd-qa-oe", "--model-path", best,
                        "--synthetic", "2"] + common, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Accuracy:" in r.stderr + r.stdout


def test_early_group_updates_match_one_update():
    """FusedAdamW.enable_early_updates: the decoder, BERT and Swin stage 4/3/2 groups are updated inside
    the backward (on the streams that finish their gradients / the decoder's weight-gradient stream)
    and the rest by step().  On the same gradients, from
    the same optimizer state, that gives the parameters of ONE update over the whole flat store, bit
    for bit."""
    from lrce.optim import FusedAdamW
    b = [t.cuda() for t in _batch("oe", 32)]
    model = _model("oe", 50, 32).cuda().train()
    opt = FusedAdamW(model, [model.parameters()], lr=1e-4, reg_strength=0.001)
    flat = opt.flat
    for _ in range(2):   # a plain first step: moments and norms become non-trivial
        opt.zero_grad()
        F.cross_entropy(model(*b[:4]).float(), b[4]).backward()
        opt.step()
    state = [t.clone() for t in (flat.f32, opt.exp_avg, opt.exp_avg_sq, opt.sumsq, opt.step_t)]
    count = opt.step_count
    opt.enable_early_updates(model.optimizer_groups())
    opt.zero_grad()
    F.cross_entropy(model(*b[:4]).float(), b[4]).backward()
    assert opt.early_updates == len(model.optimizer_groups())   # decoder, text(_hi), swin3, swin2, swin1 inside the backward
    opt.step()
    torch.cuda.synchronize()
    early = flat.f32.clone()
    # the same gradients through one whole-store update from the saved state
    for dst, src in zip((flat.f32, opt.exp_avg, opt.exp_avg_sq, opt.sumsq, opt.step_t), state):
        dst.copy_(src)
    opt.step_count = count
    opt._norm_version = flat.master_version()   # the restored norms belong to the restored weights
    opt.enable_early_updates({})
    opt.step()
    torch.cuda.synchronize()
    assert torch.equal(early, flat.f32)


def test_fp16_overflow_skips_the_text_group_update():
    """The delayed fp16 scales of BERT's backward (text.py) can overflow when a gradient grows by more
    than 2^8 between steps; the fused LN backward then raises its slot's found-inf flag and FusedAdamW's
    guard (model.overflow_guard) keeps the text group's parameters and moments for that step, as the
    reference's GradScaler skips an overflowing step (agent_oe.py:40-42), while the decoder and Swin
    groups update.  The overflow is forced by recording a tiny max in the slot of the first fp16 operand
    the backward writes (the top layer's FFN output gradient), so its next scale is 2^100; the slots
    below it see the non-finite gradient as a non-finite max and back off.  The step after it rescales
    and updates the text group again."""
    from lrce.optim import FusedAdamW
    b = [t.cuda() for t in _batch("oe", 32)]
    model = _model("oe", 50, 32).cuda().train()
    opt = FusedAdamW(model, [model.parameters()], lr=1e-4, reg_strength=0.001)
    opt.enable_early_updates(model.optimizer_groups())
    flat = opt.flat
    (c0, c1), slots = opt._guard
    text = slice(c0 * 1024, c1 * 1024)

    def step():
        opt.zero_grad()
        loss = F.cross_entropy(model(*b[:4]).float(), b[4])
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
        return loss.item()

    step()
    step()                                                   # a delayed-scale step
    assert float(slots[..., 3].abs().sum()) == 0.0
    slots.view(torch.int32)[-1, 0, 2] = 0x01800000           # recorded max 2^-124: S = 2^(7+124) -> 2^100 cap
    before = [t.clone() for t in (flat.f32, opt.exp_avg, opt.exp_avg_sq)]
    loss = step()
    assert loss == loss
    assert float(slots[..., 3].abs().sum()) != 0.0          # the top layer's operands overflowed
    for now, was in zip((flat.f32, opt.exp_avg, opt.exp_avg_sq), before):
        assert torch.equal(now[text], was[text])
    rest = torch.ones(flat.f32.numel(), dtype=torch.bool, device=flat.f32.device)
    rest[text] = False
    assert bool(torch.isfinite(flat.f32).all())
    assert (flat.f32[rest] != before[0][rest]).float().mean().item() > 0.5
    w = flat.f32[text].clone()
    step()
    assert float(slots[..., 3].abs().sum()) == 0.0
    assert bool(torch.isfinite(flat.f32).all()) and (flat.f32[text] != w).float().mean().item() > 0.5


def test_early_updates_do_not_race_the_backward():
    """The same training step run from identical weights and optimizer state — once with the
    in-backward group updates, once with one update after the backward — with every stochastic element
    off (train mode, dropout / DropPath 0, so both runs see the same gradients): flat.grad and the
    updated masters must agree.  An early update that overlapped a backward kernel still reading its
    group's weights (the decoder's and Swin stages' updates run on the weight-gradient stream, BERT's
    on the text stream), or that read a gradient before its last writer, shifts that gradient by a
    whole update step (relative ~1e-3 at lr 1e-4); the backward's own run-to-run noise (a few float
    atomics: embedding rows, bias sums of split-K weight gradients) is ~1e-7, measured here as the
    difference between two plain runs.  The test above cannot see a race: it reuses the racing run's
    gradients."""
    from lrce.optim import FusedAdamW
    b = [t.cuda() for t in _batch("oe", 32)]
    model = _model("oe", 50, 32)
    model.fusion_model.drop_out_rate = 0.0
    model.fusion_model.fusion_transformer.drop_out_rate = 0.0
    for layer in model.video_extractor.swin.layers:
        for blk in layer.blocks:
            blk.drop_path = 0.0
    model.text_extractor.bert.hidden_dropout = model.text_extractor.bert.attention_dropout = 0.0
    model = model.cuda().train()
    opt = FusedAdamW(model, [model.parameters()], lr=1e-4, reg_strength=0.001)
    flat = opt.flat
    for _ in range(2):
        opt.zero_grad()
        F.cross_entropy(model(*b[:4]).float(), b[4]).backward()
        opt.step()
    torch.cuda.synchronize()
    # BERT's delayed per-tensor gradient scales (the previous backward's maxima) are step state too:
    # restored with the rest, every run scales its fp16 gradients alike
    bufs = (flat.f32, opt.exp_avg, opt.exp_avg_sq, opt.sumsq, opt.step_t,
            model.text_extractor.bert._grad_scales(flat.device))
    state = [t.clone() for t in bufs]
    count = opt.step_count
    w0 = flat.f32.clone()

    def run(groups):
        for dst, src in zip(bufs, state):
            dst.copy_(src)
        opt.step_count = count
        flat.masters_written()                       # re-cast the bf16 / fp16 shadows of the restored masters
        opt._norm_version = flat.master_version()    # the restored norms belong to the restored weights
        opt.enable_early_updates(groups)
        n0 = opt.early_updates
        opt.zero_grad()
        F.cross_entropy(model(*b[:4]).float(), b[4]).backward()
        opt.step()
        torch.cuda.synchronize()
        return flat.grad.clone(), flat.f32.clone(), opt.early_updates - n0

    def worst(a, b_, ref):
        """max over tensors of max|a - b| / max|ref| (ref: the gradient, or the update w - w0)"""
        out = []
        for name, p in model.named_parameters():
            if not p.requires_grad:
                continue
            da = (flat._slice(a, p) - flat._slice(b_, p)).abs().max().item()
            out.append((da / (flat._slice(ref, p).abs().max().item() + 1e-30), name))
        return max(out)

    g_plain, w_plain, n_plain = run({})
    g_plain2, w_plain2, _ = run({})
    g_early, w_early, n_early = run(model.optimizer_groups())
    assert n_early == len(model.optimizer_groups()) and n_plain == 0
    noise = worst(g_plain2, g_plain, g_plain)
    err = worst(g_early, g_plain, g_plain)
    assert noise[0] < 1e-4, f"plain runs differ: {noise}"
    assert err[0] < max(1e-4, 4 * noise[0]), f"gradients with early updates: {err} (plain-run noise {noise})"
    upd = w_plain - w0
    werr = worst(w_early, w_plain, upd)
    wnoise = worst(w_plain2, w_plain, upd)
    assert werr[0] < max(1e-3, 4 * wnoise[0]), f"updates with early updates: {werr} (noise {wnoise})"


def test_capture_joins_a_forked_branch():
    """graph.py's capture guard (the r5ab2 analysis): a branch forked into the capture and
    never joined by the captured code is joined by the capture itself (runtime.join_capture_branches),
    so the capture ends cleanly and the replay runs the branch's work before the graph completes."""
    from lrce import runtime as R
    from lrce.graph import CapturedStep
    dev = torch.device("cuda", 0)
    x = torch.ones(1 << 20, device=dev)
    out = torch.zeros_like(x)
    s = R.aux_stream(dev, "grad_zero")

    def fn():
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            torch.mul(x, 2.0, out=out)      # forked, not joined here
        return out
    step = CapturedStep(fn, warmup=1)
    x.fill_(3.0)
    out.zero_()
    step.replay()
    torch.cuda.synchronize()
    assert torch.all(out == 6.0)
