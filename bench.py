#!/usr/bin/env python
"""bench.py — LRCE training-step throughput on MI355X (QA-samples/s, fwd+bwd).

One step = the reference's train_ddp.py step (agent_oe.py:19-48) on a synthetic MSVD-QA batch:
E2EOpenEnded forward (Video Swin-B 3D on 3 clips x 5 frames x 224^2 -> BERT-base on a 20-token
question padded to 32 -> 3-step x 12-layer recurrent LRCE decoder -> 1000-way head), cross-entropy,
backward, gradient all-reduce (N>1: bf16 RCCL buckets after the replayed backward), and the fused
AdamW step with the L2 regulariser (reg 0.001) over all 312 M parameters, replayed from HIP graphs by
the same TrainStepGraph the train_ddp.py agent uses.  Train mode: dropout 0.5 in the fusion model
(train_ddp default drop-out-rate), BERT dropout 0.1, Swin DropPath 0.2.  Inputs resident in HBM
before the timed region.  bf16 MFMA compute (fp16 for the BERT forward, like the reference's fp16
autocast) with f32 master weights / residual stream.  The agent path itself (pinned host batches,
process_data) is timed after the main measurement and reported as `agent_path`.

    python bench.py [--gpus N --steps K --warmup W]
N>1: one process per GPU over RCCL (the reference's train_ddp.py:136-138 spawns world_size =
device_count processes); each rank runs bs=10 (weak scaling); rank 0 prints ONE JSON line.  Started
by torch.distributed.run (WORLD_SIZE set) it is one of the ranks; started plainly with --gpus N > 1 it
first launches the N ranks itself, as children through torch.distributed.run, before anything touches
the GPU, and exits with their status.  A joined world that differs from --gpus is an error.
--dry-run: the same launcher and rank/world checks over gloo on the CPU (no model, no GPU) — the
launcher's test.
--shared-device (test-only rehearsal, never a measurement): the N ranks all run on cuda:0 and exchange
over gloo instead of RCCL, so the N-GPU model path (split backward at SPLIT_SWIN_STAGE, bf16 gradient
buckets, the early-update graphs) runs end to end on a one-GPU box; the JSON line says so.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "vqa-lrce-kbs-2023_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0      # MI355X_MICROARCH.md: ~2.5 PF dense bf16
METRIC = "QA-samples/sec (fwd+bwd) at bs=10\u00d716f\u00d7224\u00b2, 1/2/4/8 MI355X; Swin-attn MFMA%"  # BASELINE.json
STEP_GFLOP_PER_SAMPLE = 933.3       # fwd+bwd, msvd-qa-oe, temporal scale 3 (flop_counter)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every CPU this process may run on")
    ap.add_argument("--mode", choices=["graph", "eager"], default="graph",
                    help="graph: the step replayed from HIP graphs (lrce/graph.TrainStepGraph, the agent's "
                         "step; N>1: graph(fwd+bwd, bf16 bucket casts) -> RCCL bucket all-reduce -> "
                         "graph(optimizer)); eager: launched from Python, all-reduce overlapped with backward")
    ap.add_argument("--grad-reduce-dtype", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--agent-steps", type=int, default=6, help="steps of the train_ddp agent path (0: skip)")
    ap.add_argument("--roofline-steps", type=int, default=2)
    ap.add_argument("--gemm-table", default=None,
                    help="write the per-shape roofline table of the bf16 GEMMs of the roofline steps (markdown) here")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check: N gloo ranks on the CPU time an all-reduce 'step'; no GPU, no model")
    ap.add_argument("--shared-device", action="store_true",
                    help="test-only rehearsal of N > 1: every rank on cuda:0, gloo instead of RCCL (not a measurement)")
    return ap.parse_args()


def lrce_env():
    """Every LRCE_* variable set in this process's environment (the product's A/B switches): recorded
    in the JSON line, so a number measured with a non-default switch says so."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("LRCE_")}


def refuse_tampering():
    """The headline must be the full training step: refuse any LRCE_DEV_* variable (dev-only
    experiments that skip work; none is read by the product any more, but an old tree or a stray
    export must never produce a silently inflated number)."""
    bad = sorted(k for k in os.environ if k.startswith("LRCE_DEV_"))
    if bad:
        log(f"refusing to run: dev-only work-skipping variables set: {', '.join(bad)}")
        sys.exit(2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """--gpus N > 1 from a plain start: N rank processes through torch.distributed.run, as CHILDREN of
    this process, which has not touched the GPU (torch.cuda.device_count() does not initialise HIP on
    this image; nothing else here runs before this point).  Returns their exit status."""
    if not args.dry_run and not args.shared_device:
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            log(f"--gpus {args.gpus}: only {ndev} device(s) visible")
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # the host driver supports dmabuf IPC only
    log(f"launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.call(cmd, env=env)


def dry_run(args, world, rank):
    """The launcher's check on the CPU: gloo ranks, barrier + max-over-ranks timing of K all-reduce
    'steps' of a 1 MB gradient stand-in, rank 0 prints the JSON line with the joined world size."""
    x = torch.ones(1 << 18)
    for _ in range(args.warmup):
        dist.all_reduce(x)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dist.all_reduce(x)
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "value": round(world * args.batch_size * args.steps / elapsed, 3),
                          "unit": "launcher-check steps/s (not a measurement)", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
                          "config": {"parallelism": f"dp{world}", "per_gpu_batch": args.batch_size,
                                     "grad_reduce": args.grad_reduce_dtype if world > 1 else None},
                          "lrce_env": lrce_env()}), flush=True)


def replica_digest(model):
    """Two integer sums over the bits of the rank's f32 master weights (plain and position-weighted,
    wrapping int64): equal on every rank iff the replicas are (practically) bit-identical."""
    from lrce.runtime import flat_of
    v = flat_of(model).f32.view(torch.int32).long()
    w = torch.arange(v.numel(), device=v.device) % 65521 + 1
    d = torch.stack([v.sum(), (v * w).sum()])
    del v, w
    return d


def synthetic_batch(batch, seed):
    """msvd-qa-oe item contract: clips U[0,1) (16 frames -> 3 clips x 5), 20-token questions."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    clips = torch.rand(batch, 3, 5, 3, 224, 224, generator=g)
    ids = torch.zeros(batch, 32, dtype=torch.int64)
    ids[:, 0], ids[:, 19] = 101, 102
    ids[:, 1:19] = torch.randint(1000, 30522, (batch, 18), generator=g)
    mask = (ids != 0).long()
    types = torch.zeros_like(ids)
    labels = torch.randint(0, 1000, (batch,), generator=g)
    return clips, ids, mask, types, labels


def build(batch, device, grad_dtype, seed=0):
    from lrce.models.e2e import E2EOpenEnded
    from lrce.optim import FusedAdamW
    from lrce.runtime import prepare
    torch.manual_seed(seed)
    # msvd-qa-oe config (configs/msvd-qa-oe.json): feature 768, 1000 answers, text_seq_len 32,
    # video_feature_dim 1024; train_ddp defaults: drop-out-rate 0.5, temporal-scale [3].  Random init
    # (no checkpoints offline): swin_ckpt / bert_dir None.
    model = E2EOpenEnded(768, 1000, 0.5, (7, 7), 1024, 5, [3], 32, swin_ckpt=None, bert_dir=None).to(device).train()
    prepare(model)
    reducer = None
    if dist.is_initialized() and dist.get_world_size() > 1:
        from lrce.distributed import attach
        reducer = attach(model, bucket_mb=64, grad_dtype=grad_dtype)
    lr = 5e-6  # args.py default --lr, expanded to 3 groups (args.py:110-111)
    opt = FusedAdamW(model, [{"params": model.fusion_model.parameters(), "lr": lr},
                             {"params": model.text_extractor.parameters(), "lr": lr},
                             {"params": model.video_extractor.parameters(), "lr": lr}],
                     lr=lr, betas=(0.9, 0.999), reg_strength=0.001)
    if reducer is None and os.environ.get("LRCE_EARLY_UPDATES", "1") != "0":
        # single process: the decoder / BERT updates overlap the Swin backward (env 0: A/B switch)
        opt.enable_early_updates(model.optimizer_groups())
    rank = dist.get_rank() if dist.is_initialized() else 0
    batch_dev = tuple(t.to(device) for t in synthetic_batch(batch, 1000 + rank))
    return model, opt, reducer, batch_dev


def train_step(model, opt, reducer, batch):
    clips, ids, mask, types, labels = batch
    out = model(clips, ids, mask, types)
    loss = F.cross_entropy(out, labels, ignore_index=-100)
    loss.backward()
    if getattr(model, "split_backward", False):   # (set by make_step's graph modes) the extractors' part
        model.backward_extractors()
    scale = reducer.finish() if reducer is not None else 1.0
    opt.step(grad_scale=scale)
    opt.zero_grad()
    return loss


def make_step(model, opt, reducer, batch, mode, world):
    from lrce.graph import TrainStepGraph
    if mode == "eager":
        return lambda: train_step(model, opt, reducer, batch)

    def body(clips, ids, mask, types, labels):
        opt.zero_grad(overlap=True)      # the gradient clear runs beside the forward
        loss = F.cross_entropy(model(clips, ids, mask, types), labels, ignore_index=-100)
        opt.grad_ready()
        loss.backward()
        return loss.detach()
    tail = None
    if reducer is not None:
        # data parallel: split backward — the fusion head's buckets are exchanged while the extractors'
        # backward replays, BERT's and Swin stages 3-4's while Swin stages 1-2 replay
        from lrce.agent.agent_base import SPLIT_SWIN_STAGE
        model.split_backward = True
        model.split_swin_stage = SPLIT_SWIN_STAGE
        tail = model.backward_segments()
    step = TrainStepGraph(body, opt, reducer, world, tail=tail)
    return lambda: step(*batch)


def agent_path(args, device, world, rank):
    """The train_ddp.py path itself (lrce/cli.py -> AgentOE.process_data): pinned host batches from
    an in-memory loader, H2D copies overlapped with the previous step, the agent's graph-replayed step,
    device-side metrics.  Returns (QA-samples/s over all ranks, ms per step)."""
    import argparse as _ap
    from lrce.agent import AgentOE
    from lrce.models.e2e import E2EOpenEnded
    torch.manual_seed(1)
    model = E2EOpenEnded(768, 1000, 0.5, (7, 7), 1024, 5, [3], 32, swin_ckpt=None, bert_dir=None)
    a = _ap.Namespace(lr=[5e-6] * 3, reg_strength=0.001, lr_decay_factor=0.5, patience=0.5, min_lr=1e-8,
                      use_cosine_scheduler=False, dataset="msvd-qa-oe", log_dir="/tmp", epoch=1, ckpt_interval=1,
                      debug_mode=True, grad_reduce_dtype=args.grad_reduce_dtype, log_interval=50)
    agent = AgentOE(model, device.index, a, log_enabled=False, rank=rank)
    batches = [tuple(t.pin_memory() for t in synthetic_batch(args.batch_size, 2000 + 17 * rank + i)) for i in range(4)]
    warm = 2                      # eager step + capture
    loader = [batches[i % len(batches)] for i in range(warm + args.agent_steps)]
    gen = agent.process_data(loader, True, 0)
    for _ in range(warm):
        next(gen)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.agent_steps):
        next(gen)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    for _ in gen:   # the pass's end-of-epoch reduce (outside the timed region)
        pass
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    del agent, model
    torch.cuda.empty_cache()
    return world * args.batch_size * args.agent_steps / dt, 1000.0 * dt / args.agent_steps


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(threads, batch=10):
    """CPU leg: the oracle (oracle/lrce_oracle.py, the fp32 PyTorch restatement of the reference
    pinned by tests/golden) on the host cores, same workload shape: a cold training step at batch 2
    (thread pool / allocator warm-up, not reported), then ONE warm training step at the config's batch
    (forward, CE + L2 loss, backward, AdamW; no dropout) and one eval forward at that batch.
    Checker/baseline only: nothing here runs on the product path."""
    from oracle import lrce_oracle as O
    from lrce.models.e2e import E2EOpenEnded
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    tmpl = E2EOpenEnded(768, 1000, 0.5, (7, 7), 1024, 5, [3], 32, swin_ckpt=None, bert_dir=None)
    sd = {k: (v.detach().clone().requires_grad_(True) if v.is_floating_point() else v)
          for k, v in tmpl.state_dict().items()}
    del tmpl
    params = [v for v in sd.values() if v.requires_grad]
    opt = torch.optim.AdamW(params, lr=5e-6, weight_decay=0.01)

    def train(b, seed):
        clips, ids, mask, types, labels = synthetic_batch(b, seed)
        t0 = time.perf_counter()
        out = O.e2e_forward(sd, clips, ids, mask, types, "oe")
        loss = F.cross_entropy(out, labels) + 0.001 * O.l2_reg(params)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return time.perf_counter() - t0
    train(2, 7)
    dt_train = train(batch, 8)
    clips, ids, mask, types, _ = synthetic_batch(batch, 9)
    with torch.no_grad():
        t0 = time.perf_counter()
        O.e2e_forward(sd, clips, ids, mask, types, "oe")
        dt_eval = time.perf_counter() - t0
    return batch / dt_train, dt_train, batch / dt_eval, dt_eval


def main():
    args = parse()
    refuse_tampering()
    if args.gpus < 1:
        log("--gpus must be >= 1")
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
            world = dist.get_world_size()
        if world != args.gpus:
            log(f"rank {rank}: joined a world of {world} ranks, --gpus {args.gpus}")
            sys.exit(3)
        if world > 1:
            dry_run(args, world, rank)
            dist.destroy_process_group()
        elif rank == 0:
            print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": 1, "config": {"parallelism": "dp1"},
                              "lrce_env": lrce_env()}), flush=True)
        return
    shared = args.shared_device and world > 1
    dev_index = 0 if shared else local
    if world > 1:
        torch.cuda.set_device(dev_index)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()
    if world != args.gpus:
        log(f"rank {rank}: joined a world of {world} ranks but --gpus {args.gpus}")
        sys.exit(3)
    device = torch.device("cuda", dev_index)
    coll = torch.device("cpu") if shared else device   # small collectives: gloo on host tensors
    from lrce import kernels as K
    from lrce import _native
    _native.lib()
    gdt = torch.bfloat16 if args.grad_reduce_dtype == "bf16" else torch.float32
    log(f"rank {rank}/{world}: building model (bs={args.batch_size})")
    model, opt, reducer, batch = build(args.batch_size, device, gdt)
    torch.cuda.reset_peak_memory_stats(device)
    step = make_step(model, opt, reducer, batch, args.mode, world)
    split_stage = getattr(model, "split_swin_stage", None) if world > 1 else None
    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log(f"warmup {i + 1}/{args.warmup}")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    replicas = None
    if world > 1:
        t = torch.tensor([elapsed], device=coll)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        d = replica_digest(model).to(coll)
        ds = [torch.empty_like(d) for _ in range(world)]
        dist.all_gather(ds, d)
        replicas = all(torch.equal(ds[0], x) for x in ds)
    loss_v = float(loss.item())
    peak_gib = torch.cuda.max_memory_allocated(device) / 2 ** 30   # warmup (eager step + capture) and replays
    samples = world * args.batch_size * args.steps
    value = samples / elapsed
    ms = 1000.0 * elapsed / args.steps
    log(f"loss {loss_v:.4f}  {value:.2f} samples/s  {ms:.1f} ms/step ({args.mode})")
    # per-kernel roofline: HIP events around every launch of the timed kernels, on their launch
    # stream, over eager steps of the same workload (a graph replay hides individual launches)
    timer = K.KernelTimer("wattn_qkv_fwd", "wattn_bwd", "gemm", "gemm_f32", detail=True)
    with timer:
        for i in range(args.roofline_steps):
            train_step(model, opt, reducer, batch)
    torch.cuda.synchronize()
    roof = _roofline(timer)
    if args.gemm_table and rank == 0 and args.roofline_steps > 0:
        _gemm_table(timer, args.roofline_steps, args.gemm_table)
    del step, model, opt, reducer, batch
    torch.cuda.empty_cache()
    agent = None
    if args.agent_steps > 0:
        try:
            v, m = agent_path(args, device, world, rank)
            agent = {"value": round(v, 3), "ms_per_step": round(m, 3), "steps": args.agent_steps,
                     "vs_graph_bench": round(v / value, 4),
                     "path": "train_ddp.py agent: AgentOE.process_data over pinned host batches (H2D overlapped), "
                             "TrainStepGraph replay, device-side metrics"}
        except Exception as e:  # the agent leg must not hide the measurement
            agent = {"value": None, "error": repr(e)[:300]}
        log(f"agent path: {agent}")

    out = {"metric": METRIC,
           "value": round(value, 3), "unit": "QA-samples/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (random-init weights, U[0,1) clips, 20-token questions)",
           "config": {"workload": "msvd-qa-oe train_ddp step: Swin-B 3D + BERT-base + LRCE-12 decoder, temporal-scale 3",
                      "global_batch": samples // args.steps, "per_gpu_batch": args.batch_size, "frames": 16,
                      "resolution": 224, "question_tokens": 20, "text_seq_len": 32,
                      "parallelism": f"dp{world}", "launch": args.mode,
                      "split_swin_stage": split_stage,
                      "grad_reduce": args.grad_reduce_dtype if world > 1 else None,
                      "precision": "bf16 MFMA (Swin, decoder memory, backward), fp16 MFMA BERT forward, "
                                   "exact-f32 decoder query side, f32 masters"},
           "loss": round(loss_v, 4),
           "model_tflops": round(STEP_GFLOP_PER_SAMPLE * value / 1000.0, 2),
           "model_mfu": round(STEP_GFLOP_PER_SAMPLE * value / 1000.0 / (MFMA_BF16_PEAK_TFLOPS * world), 4)}
    out["peak_memory_gib"] = round(peak_gib, 2)   # torch allocator peak of the measured step (graph pool included)
    out["roofline"] = roof
    if world > 1:
        out["replicas_identical"] = replicas   # the ranks' master weights after the timed steps
    if shared:
        out["rehearsal"] = "shared-device: every rank on cuda:0 over gloo — a path test, not a measurement"
    out["lrce_env"] = lrce_env()   # non-default product switches (empty for the default step)
    if agent is not None:
        out["agent_path"] = agent
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the GPU box's CPU share is OMP_NUM_THREADS (16): more threads than that oversubscribe the
        # shared host (256 threads measured 2.4x slower than 16)
        share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16
        threads = args.cpu_threads or min(len(os.sched_getaffinity(0)), share)
        log(f"cpu baseline (oracle, fp32, {threads} threads) ...")
        try:
            v, dt, ve, dte = cpu_baseline(threads, args.batch_size)
            out["cpu_baseline"] = {"value": round(v, 4), "unit": "QA-samples/s", "cores": threads, "kind": "port",
                                   "cpu": _cpu_model(),
                                   "sample": f"one warm training step (fwd+bwd+AdamW, fp32) of the CPU oracle at batch "
                                             f"{args.batch_size}: {dt:.1f} s (after a cold batch-2 step)",
                                   "eval_forward": {"value": round(ve, 4), "unit": "QA-samples/s",
                                                    "sample": f"one eval forward at batch {args.batch_size}: {dte:.1f} s"}}
        except Exception as e:  # the baseline must not hide the GPU number
            out["cpu_baseline"] = {"value": None, "error": repr(e)[:200]}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: HBM3E ~8 TB/s
RIDGE = MFMA_BF16_PEAK_TFLOPS * 1000.0 / HBM_PEAK_GBS   # 312.5 flop/B
PMC_TRAFFIC = os.path.join(REPO, "profiles", "r6_pmc_wattn_qkv_fwd.json")   # tools/pmc_traffic.py output


def _pmc_traffic():
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 --pmc passes of this
    same command (FETCH_SIZE and WRITE_SIZE in separate runs, FETCH_SIZE doubled for gfx950)."""
    try:
        with open(PMC_TRAFFIC) as f:
            d = json.load(f)
        return round(d["traffic_bytes_per_launch"]), os.path.relpath(PMC_TRAFFIC, REPO)
    except (OSError, KeyError, ValueError):
        return None, None


def _roofline(timer):
    """Roofline of the Swin window-attention kernel the north star names, which here is ONE kernel:
    the QKV projection fused with the 3D shifted-window attention (csrc/window_fused.hip).
    Algorithmic work per launch (no credit for padding): the qkv Linear
    2 * (windows * 147) * C * 3C plus QK^T + PV 4 * 147^2 * 32 per (window, head); algorithmic bytes:
    the LN1 rows read, W_qkv read, qkv (kept for the backward) and O written, bf16.  The kernel is
    MFMA-bound where its intensity passes the bf16 ridge (2.5 PF/s / 8 TB/s = 312 flop/B: stages 3-4,
    C >= 512) and HBM-bound below it (stages 1-2): `bound` follows the step's aggregate intensity over
    all 24 launches, and both fractions are reported, plus the MFMA fraction of the attention products
    alone (the part the reference runs as bmm + softmax).  Durations: HIP events around every launch
    on its stream during eager steps of the same workload (a graph replay hides launches)."""
    n, mean_ms, tflops, gbs = timer.summary("wattn_qkv_fwd")
    if not n:
        return None
    traffic, src = _pmc_traffic()
    fl, by = timer.flops["wattn_qkv_fwd"], timer.bytes["wattn_qkv_fwd"]
    ai = fl / by
    mf, hf = tflops / MFMA_BF16_PEAK_TFLOPS, gbs / HBM_PEAK_GBS
    attn_fl = sum(4.0 * 147 * 147 * 32 * key[0] * key[1] * len(ev) for (name, key), (ev, _) in timer.detail.items()
                  if name == "wattn_qkv_fwd") if timer.detail is not None else None
    total_ms = timer.total_ms("wattn_qkv_fwd")
    roof = {"kernel": "lrce_wattn_qkv_fwd (qkv Linear + window attention fused)",
            "bound": "mfma" if ai >= RIDGE else "hbm",
            "achieved": round(tflops if ai >= RIDGE else gbs, 2), "peak": MFMA_BF16_PEAK_TFLOPS if ai >= RIDGE else HBM_PEAK_GBS,
            "unit": "TFLOP/s" if ai >= RIDGE else "GB/s", "frac": round(mf if ai >= RIDGE else hf, 4),
            "traffic": traffic, "traffic_source": src,
            "algorithmic_bytes_per_launch": round(by / n), "algorithmic_flops_per_launch": round(fl / n),
            "intensity_flop_per_byte": round(ai, 1), "ridge_flop_per_byte": RIDGE,
            "launches": n, "mean_launch_ms": round(mean_ms, 4),
            "mfma_frac": round(mf, 4), "hbm_frac": round(hf, 4)}
    if attn_fl is not None and total_ms > 0:
        roof["attention_only_mfma_frac"] = round(attn_fl / total_ms / 1e9 / MFMA_BF16_PEAK_TFLOPS, 4)
    per = {}
    for (name, key), (ev, f) in (timer.detail or {}).items():
        if name == "wattn_qkv_fwd":
            t = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
            per[f"windows{key[0]}_heads{key[1]}"] = {"mean_launch_ms": round(t, 4),
                                                     "tflops": round(f / len(ev) / t / 1e9, 1)}
    roof["per_stage"] = per
    extra = {}
    for name in ("wattn_bwd", "gemm", "gemm_f32"):
        if name in timer.names:
            c, m, t, _ = timer.summary(name)
            if c:
                extra[name] = {"launches": c, "mean_launch_ms": round(m, 4), "achieved_tflops": round(t, 2),
                               "frac": round(t / MFMA_BF16_PEAK_TFLOPS, 4)}
    roof["others"] = extra
    return roof


def _gemm_table(timer, steps, path):
    """Per-shape roofline of the bf16 / fp16 MFMA GEMMs (lrce_gemm, LDS-DMA / register-staged paths) over
    the roofline steps: algorithmic flops 2 M N K and bytes (A, B once; C by its epilogue: 16-bit or
    f32 out, an f32 accumulate read, residual / pre-activation operands), the bound they imply against
    the bf16 ridge, and the fraction of that bound the launch reaches (HIP events, eager steps)."""
    from lrce import _native as N
    rows, tot_us = [], 0.0
    for name, key, calls, t_ms, tf in timer.breakdown():
        if name != "gemm":
            continue
        m, n, k, batch, al, bl, a32, split, flags = key
        ab = 4 if a32 == "a32" else 2
        outb = 4 if flags & (N.EPI_OUT_F32 | N.EPI_ATOMIC | N.EPI_ACCUM) else 2
        if flags & N.EPI_ACCUM:
            outb += 4
        outb += (4 if flags & N.EPI_RESID else 0) + (2 if flags & N.EPI_DGELU else 0) + \
            (2 if flags & N.EPI_AUX_OUT else 0) + (2 if flags & N.EPI_OUT_BOTH else 0)
        byts = batch * (ab * m * k + 2 * n * k + outb * m * n)
        fl = 2.0 * m * n * k * batch
        us = 1000.0 * t_ms / calls
        ai = fl / byts
        bound = "mfma" if ai >= RIDGE else "hbm"
        ach_tf, ach_gb = fl / us / 1e6, byts / us / 1e3
        frac = ach_tf / MFMA_BF16_PEAK_TFLOPS if bound == "mfma" else ach_gb / HBM_PEAK_GBS
        per_step_us = 1000.0 * t_ms / steps
        tot_us += per_step_us
        rows.append((per_step_us, f"| {m}x{n}x{k}{'' if batch == 1 else f' x{batch}'} | {al}/{bl}/{a32} | {split} | {flags} | "
                                  f"{calls / steps:g} | {us:.1f} | {per_step_us:.0f} | {ach_tf:.0f} | {ach_gb:.0f} | {ai:.0f} | "
                                  f"{bound} | {frac:.3f} |"))
    rows.sort(key=lambda r: -r[0])
    with open(path, "w") as f:
        f.write(f"# bf16/fp16 GEMM launches per training step (bench.py --gemm-table, {steps} eager roofline steps)\n")
        f.write(f"# total {tot_us / 1000:.2f} ms/step of lrce_gemm launches (HIP events; eager, so launch gaps excluded)\n\n")
        f.write("| M x N x K | A/B layout | split-K | epilogue flags | launches/step | us/launch | us/step | TFLOP/s | GB/s "
                "| flop/B | bound | frac of bound |\n|---|---|---|---|---|---|---|---|---|---|---|---|\n")
        for _, r in rows:
            f.write(r + "\n")


if __name__ == "__main__":
    main()
