"""Training-step parity at the BASELINE batch sizes (BASELINE.json configs 2-5): the full model's
parameter gradients on the HIP path vs the CPU oracle's autograd on the same batch.

Workloads (dropout / DropPath off, train mode, so every tile / split-K depth the bench runs at
these batch sizes is exercised — the split depth of a weight gradient depends on M = tokens):
  * msvd-qa-oe, bs 10, temporal scale 3, cross-entropy (agent_oe.py:35-36);
  * msrvtt-qa-oe, bs 10, L = 37, 1500 answers, cross-entropy (configs/msrvtt-qa-oe.json);
  * tgif-transition 5-way MC, bs 9, multi-class hinge loss (agent_mc.py:20-41, margin 1);
  * tgif-count, bs 10, L = 30, mean-squared error on the ReLU count (agent_count.py:35-44).
The L2 regulariser's gradient reg * p / ||p|| (agent_base.py:103-108) is not a model-backward
term: it is folded into the AdamW kernel and checked against torch there (test_ops_gpu.py).

Every floating-point parameter is compared (783 tensors); tensors whose oracle gradient is exactly
zero (BERT pooler, decoder self-attention q/k: softmax over one key) must be zero here too, and the
analytically-zero BERT key biases (rounding noise on both sides) small against the query biases.

Bar per tensor, as max|d| / max|ref| against the fp32 oracle — a RATCHET on the committed
measurement of this path (tests/golden/train_grad_errors.json, the round-5 GPU run): min(CAP, max(3e-2, 1.5 x the committed error)), CAP = 0.1; the
kernels are deterministic up to a few f32 atomics, so a 1.5x margin catches regressions.  For scale,
the reference's own training numerics (fp16 autocast + GradScaler, restated on the CPU in
tests/golden/make_train_yardstick.py) make at most 0.028 on any tensor of these batches, and the same
numerics in bf16 up to 0.28 (BERT top-layer query / key) / 0.08 (Swin relative-position tables); the
committed errors are <= 0.03 except the Swin relative-position tables (bf16 dS summed over ~1e5
terms; <= 0.052, tgif-transition).  Tensors absent from the committed file fall back to the yardstick
bar: 3e-2, 2x the fp16 yardstick, 2.5x the bf16 one for Swin / fusion tensors, never above CAP.
The measured errors are written to $LRCE_PARITY_OUT (JSON) when set.

test_second_train_step_grads_match_oracle checks the gradients of a training step as the bench and the
trainer run it from the second step on: BERT's delayed gradient scales (the previous step's maxima,
text._Stack.delayed) and the fresh-gradient STORE epilogues of the deferred / batched weight
gradients (FlatParams.claim_fresh after FusedAdamW.zero_grad), against the same oracle and bars.
The oracle runs on the GPU box's host cores as the checker (about 25 s / batch)."""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import load_recipe, oracle_sd, rel
from oracle import lrce_oracle as O
from oracle import weights as W

pytestmark = pytest.mark.gpu

CFG = {"msvd-qa-oe": ("oe", 1000, 32), "msrvtt-qa-oe": ("oe", 1500, 37), "tgif-transition": ("mc", 1, 40),
       "tgif-count": ("count", 1, 30)}
WORKLOADS = [("msvd-qa-oe", 10), ("msrvtt-qa-oe", 10), ("tgif-transition", 9), ("tgif-count", 10)]
SEED = 31

# max|d| / max|ref| per tensor family: bf16 GEMM operands and bf16 backward (Swin, BERT); the fusion
# gradients inherit the bf16 features (the MC head's single logit is a cancellation-heavy sum)
TOL = {"swin": 3e-2, "bert": 3e-2, "fusion": 3e-2}
YARD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "train_grad_yardstick.json")
RATCHET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "train_grad_errors.json")


def _family(name):
    if name.startswith("video_extractor."):
        return "swin"
    if name.startswith("text_extractor."):
        return "bert"
    return "fusion"


def _build(name):
    from lrce.models import e2e
    task, ncls, L = CFG[name]
    cls = {"oe": e2e.E2EOpenEnded, "mc": e2e.E2EMultipleChoice, "count": e2e.E2ECount}[task]
    return cls(768, ncls, 0.0, (7, 7), 1024, 5, [3], L)


def recipe(name):
    """(recipe state dict, task, text length) of a workload, without a GPU (the yardstick script)."""
    m = _build(name)
    filled = W.fill_state_dict({k: v for k, v in m.state_dict().items()}, 0)
    return filled, CFG[name][0], CFG[name][2]


def _model(name):
    task = CFG[name][0]
    m = _build(name)
    # train mode with every stochastic element off: DropPath (video_swin_ori.py:546), BERT dropout
    for layer in m.video_extractor.swin.layers:
        for blk in layer.blocks:
            blk.drop_path = 0.0
    m.text_extractor.bert.hidden_dropout = m.text_extractor.bert.attention_dropout = 0.0
    filled = load_recipe(m)
    return m.cuda().train(), filled, task


def _inputs(name, batch, seed):
    task, ncls, L = CFG[name]
    clips = W.synthetic_clips(batch, 3, seed=seed)
    if task == "mc":
        ids, mask, types = W.synthetic_question(batch, L, seed=seed, n_choice=5, ans_tokens=8)
        label = torch.from_numpy(np.random.default_rng(seed).integers(0, 5, size=batch))
    elif task == "count":
        ids, mask, types = W.synthetic_question(batch, L, seed=seed)
        label = torch.from_numpy(np.random.default_rng(seed).integers(1, 8, size=batch).astype(np.float32))
    else:
        ids, mask, types = W.synthetic_question(batch, L, seed=seed)
        label = torch.from_numpy(np.random.default_rng(seed).integers(0, ncls, size=batch))
    return clips, ids, mask, types, label


def _loss(task, out, label):
    """The agents' task losses: hinge (agent_mc.py:20-41, margin 1), mean MSE (agent_count.py:35-44),
    cross-entropy (agent_oe.py:35-36)."""
    if task == "mc":
        from lrce.agent.agent_mc import hinge_loss
        return hinge_loss(out, label, 1.0)
    if task == "count":
        return F.mse_loss(out.float(), label.float())
    return F.cross_entropy(out.float(), label, ignore_index=-100)


def oracle_loss(task, y, label):
    if task == "mc":
        return O.hinge_loss(y, label, 1.0)
    if task == "count":
        return F.mse_loss(y, label.float())
    return F.cross_entropy(y, label, ignore_index=-100)


CAP = 0.1
# The bf16 yardstick of a tensor is ONE sample of a rounding process (the same tensor role in the
# neighbouring blocks spans 0.017-0.05 for the stage-3 relative-position tables): the measured errors
# sit at 0.7-1.1x it, the largest ratio over the four batches is 2.06x (one stage-3 table).
BF16_FACTOR = 2.5


def _allow(tol, y, fam, committed=None):
    """The bar of one tensor (module docstring): the ratchet on its committed error, else the
    yardstick bar; never above CAP."""
    if committed is not None:
        return min(CAP, max(tol, 1.5 * committed))
    b = max(tol, 2.0 * y.get("fp16", 0.0))
    if fam in ("swin", "fusion"):
        b = max(b, BF16_FACTOR * y.get("bf16", 0.0))
    return min(CAP, b)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(m, name, batch, task, seed):
    clips, ids, mask, types, label = _inputs(name, batch, seed=seed)
    y = m(clips.cuda(), ids.cuda(), mask.cuda(), types.cuda())
    loss = _loss(task, y, label.cuda())
    loss.backward()
    torch.cuda.synchronize()
    return y, loss


@pytest.mark.parametrize("name,batch", WORKLOADS)
def test_baseline_train_step_grads_match_oracle(name, batch):
    m, filled, task = _model(name)
    m.zero_grad(set_to_none=True)
    y, loss = _run(m, name, batch, task, SEED)
    _check_against_oracle(m, filled, name, batch, task, y, loss, "")


@pytest.mark.parametrize("name,batch", WORKLOADS)
def test_second_train_step_grads_match_oracle(name, batch):
    """The default training path of every step after the first: a warm-up backward on
    another batch records BERT's gradient maxima (its scales are then delayed ones), then the
    optimizer's zero_grad arms the fresh-gradient STORE epilogues, and the second backward's gradients
    must meet the first step's bars.  No optimizer step runs, so the masters are the oracle's."""
    from lrce.optim import FusedAdamW
    from lrce.runtime import flat_of
    m, filled, task = _model(name)
    opt = FusedAdamW(m, [m.parameters()], lr=1e-4)
    opt.zero_grad()
    _run(m, name, batch, task, SEED + 1)
    assert getattr(m.text_extractor.bert, "_lrce_scales_ready", False), "no delayed scales after a full backward"
    opt.zero_grad()
    flat = flat_of(m)
    claims = []
    orig = flat.claim_fresh

    def claim(params):
        r = orig(params)
        claims.append(r)
        return r
    flat.claim_fresh = claim
    try:
        y, loss = _run(m, name, batch, task, SEED)
    finally:
        flat.claim_fresh = orig
    # (a parameter claimed twice in one backward — the decoder's in_proj rows, Q then K/V — accumulates
    # the second time; most claims must be fresh)
    assert claims and 2 * sum(claims) > len(claims), f"STORE path not taken: {sum(claims)} of {len(claims)} claims fresh"
    print(f"\n{sum(claims)} of {len(claims)} weight-gradient claims fresh (STORE)")
    _check_against_oracle(m, filled, name, batch, task, y, loss, "_step2")


def _check_against_oracle(m, filled, name, batch, task, y, loss, tag):
    grads = {k: p.grad.detach().float().cpu() for k, p in m.named_parameters() if p.grad is not None}
    y = y.detach().float().cpu()
    loss = float(loss.detach())
    del m
    torch.cuda.empty_cache()
    clips, ids, mask, types, label = _inputs(name, batch, seed=SEED)
    torch.set_num_threads(min(16, torch.get_num_threads()))
    sd = oracle_sd(filled, requires_grad=True)
    yr = O.e2e_forward(sd, clips, ids, mask, types, task)
    lr_ = oracle_loss(task, yr, label)
    lr_.backward()
    if task == "count":
        assert int((yr > 0).sum()) >= batch // 2, "count head: too few positive outputs for a gradient test"
    assert rel(y, yr) < 1e-2
    lr_v = float(lr_.detach())
    assert abs(loss - lr_v) < 1e-2 * max(1.0, abs(lr_v))

    with open(YARD) as f:
        yard = json.load(f)[f"{name}_b{batch}"]
    with open(RATCHET) as f:
        ratchet = json.load(f).get(f"{name}_b{batch}", {})
    worst = {f: (0.0, "") for f in TOL}
    errs, bad = [], []
    record = {}
    checked = 0
    for k, t in sd.items():
        if not t.is_floating_point():
            continue
        assert k in grads, f"no gradient for {k}"
        g, gr = grads[k], t.grad
        if gr is None or float(gr.abs().max()) == 0.0:
            # exactly-zero reference gradient (unused pooler, one-key softmax q/k): ours ~0 too
            assert float(g.abs().max()) < 1e-6, (k, float(g.abs().max()))
            continue
        if k.endswith("attention.self.key.bias"):
            # analytically zero (a key bias shifts every logit of a softmax row by the same q.b):
            # both sides are rounding noise; bound ours by the query-bias gradient's scale
            qb = sd[k.replace("key.bias", "query.bias")].grad
            kb = float(g.abs().max()) / float(qb.abs().max())
            kbar = _allow(2e-2, yard.get(k, {}), "bert", ratchet.get(k))
            record[k] = {"err": round(kb, 6), "bar": round(kbar, 6), **yard.get(k, {})}
            if kb > kbar:
                bad.append((kb, kbar, k))
            continue
        e = rel(g, gr)
        fam = _family(k)
        bar = _allow(TOL[fam], yard.get(k, {}), fam, ratchet.get(k))
        errs.append((e, bar, k))
        record[k] = {"err": round(e, 6), "bar": round(bar, 6), **yard.get(k, {})}
        if e > bar:
            bad.append((e, bar, k))
        if e > worst[fam][0]:
            worst[fam] = (e, k)
        checked += 1
    print(f"\n{name} bs{batch}{tag}: {checked} tensors; worst per family: {worst}")
    for e, bar, k in sorted(errs, reverse=True)[:40]:
        print(f"  {e:.3e} (bar {bar:.3e})  {k}")
    n_yard = sum(1 for e, bar, k in errs if e > TOL[_family(k)])
    print(f"  {n_yard} tensors above 3e-2, within their yardstick bar (<= {CAP})")
    out = os.environ.get("LRCE_PARITY_OUT")
    if out:
        allrec = json.load(open(out)) if os.path.exists(out) else {}
        allrec[f"{name}_b{batch}{tag}"] = {"loss": loss, "loss_ref": lr_v, "logits_rel": rel(y, yr), "tensors": record}
        with open(out, "w") as f:
            json.dump(allrec, f, indent=0, sort_keys=True)
    assert checked > 500
    assert not bad, bad
