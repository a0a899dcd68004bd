"""Training / evaluation agent (reference lrce/agent/agent_base.py) on the native gfx950 path.

Same class name, constructor `(model, gpu_id, args, log_enabled=True, is_eval=False)`, attributes
(`model` with `.module`, `optim`, `scheduler`, `args`, `last_loss`, `last_metric_val`, `best_*`) and
methods (`step`, `process_data` generator, `do_training`, `do_sanity_check`, `do_evaluation`,
`save_checkpoint` / `load_checkpoint` with the `{'model_state_dict': ...}` format,
`calculate_l2_reg`, `is_metric_val_better`, `save_config`, `write_summary`).

What differs, MI355X-first:
* optimizer: FusedAdamW over the flat parameter store, three groups (fusion, text, video) with the
  per-group learning rates of args.lr (agent_base.py:27-44).  The loss's L2 term
  reg_strength * sum_t ||p_t||_2 (agent_base.py:103-108) is not back-propagated through 783 norm
  kernels: its gradient reg * p_t / ||p_t|| is added inside the update kernel, and its value comes
  from the norms that kernel already produces — the reported loss is the reference's loss;
* precision: bf16 MFMA with f32 master weights instead of fp16 autocast + GradScaler (no loss scale is
  needed for bf16; `self.scaler` is kept as None);
* data parallel: instead of torch DDP (agent_base.py:75-76), `DataParallel` below attaches the
  bucketed RCCL gradient reducer of lrce/distributed.py (bf16 buckets by default, eager: all-reduce
  overlapped with backward; 1/world folded into the optimizer's gradient scale, one parameter
  broadcast at construction);
* launch: a training step is replayed from HIP graphs (lrce/graph.TrainStepGraph: the first batch of
  a shape runs eagerly, the next one is captured) — the same step bench.py times; `args.eager = True`
  (CLI --eager) keeps Python-launched steps;
* no per-step host syncs: the batch loss / metric stay on the device; the per-step summaries are
  read back every `log_interval` steps (same tags and step indices) and the epoch metric is reduced
  to rank 0 once per pass instead of after every batch (same value: sum over ranks and batches);
* summaries: tensorboard is not in this image; scalars go to `<log_dir>/scalars.jsonl` (same tags).
"""
import json
import logging
import os
import time
from collections import deque

import torch
import torch.distributed as dist
import torch.nn as nn

from ..graph import TrainStepGraph

# data-parallel split backward: the Swin backward is cut before this stage (E2EBase.split_swin_stage)
SPLIT_SWIN_STAGE = 2
from ..optim import FusedAdamW
from ..runtime import ensure
from .schedulers import CosineAnnealingWarmupRestarts, ReduceLROnPlateau

IGNORE_INDEX = -100   # constants.py:10


def get_logger(name, rank):
    """utils.py:163-175: a real logger on rank 0, a silent one elsewhere."""
    logger = logging.getLogger(name)
    if rank != 0:
        logger.disabled = True
    return logger


class ScalarLog:
    """Minimal stand-in for torch.utils.tensorboard.SummaryWriter.add_scalar (JSON lines)."""

    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, "scalars.jsonl")

    def add_scalar(self, tag, value, step):
        with open(self.path, "a") as f:
            f.write(json.dumps({"tag": tag, "value": float(value), "step": step}) + "\n")


class DataParallel(nn.Module):
    """The agent's replacement for DistributedDataParallel: `.module` is the model; when a process
    group with more than one rank exists, gradients are averaged by the flat-buffer RCCL reducer."""

    def __init__(self, module, bucket_mb=64, grad_dtype=torch.bfloat16):
        super().__init__()
        self.module = module
        self.reducer = None
        ensure(module)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            from ..distributed import attach
            self.reducer = attach(module, bucket_mb=bucket_mb, grad_dtype=grad_dtype)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def finish_gradients(self):
        """Wait for the all-reduce of every bucket; returns the optimizer's gradient scale (1/world)."""
        return self.reducer.finish() if self.reducer is not None else 1.0


class AgentBase:
    def __init__(self, model, gpu_id, args, log_enabled=True, is_eval=False, rank=None):
        """gpu_id: this process's device (LOCAL_RANK); rank: its global rank (default: the process
        group's rank, else gpu_id) — rank 0 logs and writes checkpoints."""
        self.args = args
        self.gpu_id = gpu_id
        if rank is None:
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else gpu_id
        self.rank = rank if isinstance(rank, int) else 0
        self.log_interval = int(getattr(args, "log_interval", 50))
        self.use_graph = not getattr(args, "eager", False)
        self._graph = None
        self.log_enabled = log_enabled
        self.is_eval = is_eval
        self.uid = int(time.time())
        self.device = torch.device("cuda", gpu_id) if isinstance(gpu_id, int) else torch.device(gpu_id)
        self.loss_func = nn.CrossEntropyLoss(ignore_index=IGNORE_INDEX)
        self.scaler = None

        model = model.to(self.device)
        gdt = torch.float32 if getattr(args, "grad_reduce_dtype", "bf16") == "f32" else torch.bfloat16
        self.model = DataParallel(model, grad_dtype=gdt)
        self.reg_strength = float(getattr(args, "reg_strength", 0.0))
        self.optim = None
        self.scheduler = None
        if not is_eval:
            lrs = list(args.lr) * (3 if len(args.lr) == 1 else 1)
            self.optim = FusedAdamW(
                model,
                [{"params": model.fusion_model.parameters(), "lr": lrs[0]},
                 {"params": model.text_extractor.parameters(), "lr": lrs[1]},
                 {"params": model.video_extractor.parameters(), "lr": lrs[2]}],
                lr=lrs[0], betas=(0.9, 0.999), reg_strength=self.reg_strength)
            if self.model.reducer is None and hasattr(model, "optimizer_groups"):
                # single process: decoder / BERT updates overlap the Swin backward
                self.optim.enable_early_updates(model.optimizer_groups())
            if getattr(args, "use_cosine_scheduler", False):
                self.scheduler = CosineAnnealingWarmupRestarts(
                    self.optim, first_cycle_steps=args.lr_restart_epoch, cycle_mult=args.lr_restart_mul,
                    max_lr=lrs[0], min_lr=args.min_lr, warmup_steps=args.lr_warm_up, gamma=args.lr_decay_factor)
            else:
                self.scheduler = ReduceLROnPlateau(self.optim, mode="max", factor=args.lr_decay_factor,
                                                   patience=args.patience, min_lr=args.min_lr)

        self.logger = get_logger(__name__, self.rank)
        self.summary_writer = None
        if log_enabled and self.rank == 0:
            self.args.log_dir = os.path.join(args.log_dir, f"{self.uid}_{args.dataset}")
            self.summary_writer = ScalarLog(self.args.log_dir)
            self.args.ckpt_dir = os.path.join(self.args.log_dir, "weights")
            os.makedirs(self.args.ckpt_dir, exist_ok=True)
            self.save_config()

        self.last_loss = None
        self.last_metric_val = None
        self.counter = 0
        self.best_epoch = None
        self.best_metric_val = None

    # ------------------------------------------------------------------ task hooks
    # A task agent supplies: the loss (task_loss), what step() returns (pack_step) and how a step's
    # result feeds the epoch metric (unpack_step -> (loss, numerator, denominator)); METRIC names the
    # summary tag and HIGHER_IS_BETTER the direction (best checkpoint, plateau scheduler).
    METRIC = "Accuracy"
    HIGHER_IS_BETTER = True

    def task_loss(self, out, gt):
        return self.loss_func(out, gt)

    def pack_step(self, loss_value, out, gt, task_terms):
        """step()'s return value (agent_oe.py:44-48): (loss, correct, total)."""
        num, den = self.metric_terms(out, gt, task_terms)
        return loss_value, int(num.item()), den

    def metric_terms(self, out, gt, task_terms):
        """(numerator as a device scalar, denominator) of the epoch metric for one batch."""
        prediction = torch.argmax(out, dim=1)
        return torch.sum(prediction == gt), prediction.shape[0]

    def unpack_step(self, result):
        return result

    # ------------------------------------------------------------------ helpers (agent_base.py:90-108)
    def is_metric_val_better(self, epoch=None):
        last, best = self.last_metric_val, self.best_metric_val
        if best is None or (last > best if self.HIGHER_IS_BETTER else last < best):
            self.best_metric_val, self.best_epoch = last, epoch
            return True
        return False

    def write_summary(self, title, value, step):
        if self.summary_writer is not None:
            self.summary_writer.add_scalar(title, value, step)

    def calculate_l2_reg(self):
        """sum over trainable parameters of ||p||_2 (device scalar, no autograd graph)."""
        if self.optim is not None:
            return self.optim.l2_value()
        with torch.no_grad():
            return sum(p.float().norm(2) for p in self.model.module.parameters() if p.requires_grad)

    def _train_body(self, video_clips, texts, texts_attention_mask, texts_type_ids, gt):
        """Forward, task loss, L2 value of the current weights, backward (no optimizer step): the
        part of agent_oe.py:27-40 a HIP graph captures.  Returns device tensors."""
        self.optim.zero_grad(overlap=True)   # the gradient clear runs beside the forward
        out = self.model(video_clips, texts, texts_attention_mask, texts_type_ids)
        terms = self.task_loss(out.float(), gt)
        task = terms.mean() if terms.dim() else terms
        l2 = self.calculate_l2_reg() if self.reg_strength != 0.0 else None
        self.optim.grad_ready()
        task.backward()
        return out.detach(), terms.detach(), task.detach(), l2

    def _step_dev(self, video_clips, texts, texts_attention_mask, texts_type_ids, ground_truth, is_train):
        """One batch on the device: (reported loss, logits, labels, per-sample loss terms), all device
        tensors (no host sync).  Training: zero_grad -> forward -> backward -> (all-reduce) -> fused
        AdamW, replayed from HIP graphs unless args.eager.  Only the task loss is back-propagated:
        the optimizer kernel adds the L2 term's gradient reg * p / ||p||."""
        d = self.device
        if is_train:
            inputs = (video_clips, texts, texts_attention_mask, texts_type_ids, ground_truth)
            if self.use_graph:
                if self._graph is None:
                    red = self.model.reducer
                    tail = None
                    mod = self.model.module
                    if red is not None and hasattr(mod, "backward_segments"):
                        # data parallel: the head's gradient buckets are exchanged while the
                        # extractors' backward replays, and BERT's + Swin stages 3-4's while Swin
                        # stages 1-2 replay (TrainStepGraph tail segments)
                        mod.split_backward = True
                        mod.split_swin_stage = SPLIT_SWIN_STAGE
                        tail = mod.backward_segments()
                    self._graph = TrainStepGraph(self._train_body, self.optim, red, red.world if red else 1, tail=tail)
                out, terms, task, l2 = self._graph(*inputs)
                gt = self._graph.static[4]
            else:
                inputs = [t.to(d, non_blocking=True) for t in inputs]
                out, terms, task, l2 = self._train_body(*inputs)
                self.optim.step(grad_scale=self.model.finish_gradients())
                gt = inputs[4]
        else:
            out = self.model(video_clips.to(d, non_blocking=True), texts.to(d, non_blocking=True),
                             texts_attention_mask.to(d, non_blocking=True), texts_type_ids.to(d, non_blocking=True))
            gt = ground_truth.to(d, non_blocking=True)
            terms = self.task_loss(out.float(), gt)
            task = terms.mean() if terms.dim() else terms
            l2 = self.calculate_l2_reg() if self.reg_strength != 0.0 else None
            out, terms = out.detach(), terms.detach()
        value = task.detach() if l2 is None else task.detach() + self.reg_strength * l2
        return value, out, gt, terms

    def step(self, video_clips, texts, texts_attention_mask, texts_type_ids, ground_truth, is_train):
        """agent_oe.py:19-48 (and its MC / count twins): one batch, host-side results."""
        value, out, gt, terms = self._step_dev(video_clips, texts, texts_attention_mask, texts_type_ids, ground_truth,
                                               is_train)
        return self.pack_step(value.item(), out, gt, terms)

    # ------------------------------------------------------------------ loops (agent_base.py:110-171)
    def _flush(self, pend):
        """Write the buffered per-step summaries (one device->host read for all of them)."""
        if not pend:
            return
        if self.summary_writer is not None:
            vals = torch.stack([torch.stack([l.float(), n.float()]) for _, l, n, _, _ in pend]).tolist()
            for (counter, _, _, den, lrs), (loss, num) in zip(pend, vals):
                for k, lr in enumerate(lrs):
                    self.write_summary(f"LR Scheduler/{k}", lr, counter)
                self.write_summary("Training/Batch Loss", loss, counter)
                self.write_summary(f"Training/Batch {self.METRIC}", num / den, counter)
        pend.clear()

    def process_data(self, dl, is_train, epoch):
        """Generator over one pass of `dl`; in training yields each batch index (the evaluation hook
        of do_training), then -1.  Batch losses and metric terms accumulate on the device; the
        metric is reduced to rank 0 once per pass (the reference reduces after every batch: same
        sum), per-step summaries are flushed every log_interval steps."""
        phase = "Training" if is_train else "Validation"
        if is_train or not self.is_eval:
            self.logger.info(f"{phase} Phase")
        acc = torch.zeros(2, device=self.device)         # metric numerator, denominator
        losses = []
        pend = []
        for i, batch in enumerate(dl):
            self.model.train(is_train)
            with torch.set_grad_enabled(is_train):
                value, out, gt, terms = self._step_dev(*batch, is_train=is_train)
            num, den = self.metric_terms(out, gt, terms)
            num = num.detach().float().reshape(())
            acc[0] += num
            acc[1] += den
            losses.append(value.detach().float().reshape(()).clone())
            if is_train:
                self.counter += 1
                if getattr(self.args, "use_cosine_scheduler", False):
                    self.scheduler.step(epoch + i / len(dl))
                pend.append((self.counter, losses[-1], num.clone(), den, [g["lr"] for g in self.optim.param_groups]))
                if len(pend) >= self.log_interval:
                    self._flush(pend)
                yield i
        self._flush(pend)
        if dist.is_available() and dist.is_initialized():
            dist.reduce(acc, dst=0)
        avg_loss = avg_metric = float("nan")
        if losses:
            lt = torch.stack(losses)
            nz = lt != 0                                 # the reference averages the nonzero batch losses
            avg_loss = float((lt * nz).sum() / nz.sum().clamp(min=1)) if bool(nz.any()) else 0.0
            avg_metric = (acc[0] / acc[1]).item()
        if is_train:
            self.write_summary("Training/Loss", avg_loss, epoch)
            self.write_summary(f"Training/{self.METRIC}", avg_metric, epoch)
        else:
            self.last_loss, self.last_metric_val = avg_loss, avg_metric
            if not self.is_eval and not getattr(self.args, "use_cosine_scheduler", False):
                self.scheduler.step(avg_metric if self.HIGHER_IS_BETTER else -avg_metric)
            self.write_summary("Validation/Loss", avg_loss, epoch)
            self.write_summary(f"Validation/{self.METRIC}", avg_metric, epoch)
        yield -1

    # ------------------------------------------------------------------ persistence (agent_base.py:173-217)
    def save_config(self):
        if not getattr(self.args, "debug_mode", True):
            vars(self.args).pop("debug_mode", None)
        config = {**vars(self.args)}
        self.logger.info("======CONFIGURATIONS======")
        for k, v in config.items():
            self.logger.info(f"{k.upper()}: {v}")
        path = os.path.join(self.args.log_dir, "config.json")
        with open(path, "w") as f:
            json.dump(config, f)
        self.logger.info(f"Training config saved to {path}")

    def save_checkpoint(self, epoch, name="", only_model=True):
        if self.rank != 0 or not hasattr(self.args, "ckpt_dir"):
            return None   # (the reference raises AttributeError here when logging is disabled)
        ckpt = {"model_state_dict": self.model.module.state_dict()}
        if not only_model:
            ckpt["optimizer_state_dict"] = self.optim.state_dict()
            ckpt["scheduler_state_dict"] = self.scheduler.state_dict()
        if name != "":
            path = os.path.join(self.args.ckpt_dir, f"{name}.pt")
        else:
            path = os.path.join(self.args.ckpt_dir,
                                f"epoch{epoch:02}_loss{self.last_loss:.4f}_metric{self.last_metric_val:.4f}.pt")
        torch.save(ckpt, path)
        self.logger.info(f"Checkpoint saved to {path}")
        return path

    def load_checkpoint(self, ckpt_path, only_model=True):
        """Loads a reference `{'model_state_dict': ...}` checkpoint (tensors only: weights_only=True)."""
        assert os.path.exists(ckpt_path), ckpt_path
        ckpt = torch.load(ckpt_path, map_location="cpu", weights_only=True)
        self.model.module.load_state_dict(ckpt["model_state_dict"])
        if not only_model:
            self.optim.load_state_dict(ckpt["optimizer_state_dict"])
            self.scheduler.load_state_dict(ckpt["scheduler_state_dict"])
        self.logger.info(f"Succesfully loaded model in {ckpt_path}")

    # ------------------------------------------------------------------ drivers (agent_base.py:219-254)
    def do_training(self, train_dataloader, val_dataloader, eval_per_epoch=1):
        eval_idx = [len(train_dataloader) // eval_per_epoch * i for i in range(1, eval_per_epoch)]
        for i in range(self.args.epoch):
            self.logger.info(f"Epoch {i + 1}/{self.args.epoch}")
            k = 0
            for step in self.process_data(train_dataloader, True, i):
                if step in eval_idx or step == -1:
                    deque(self.process_data(val_dataloader, False, eval_per_epoch * i + k), maxlen=0)
                    if self.is_metric_val_better(i + 1):
                        self.save_checkpoint(i + 1, "best")
                    k += 1
            if (i + 1) % self.args.ckpt_interval == 0 or i == self.args.epoch - 1:
                self.save_checkpoint(i + 1)
            self.logger.info("Epoch complete\n")
        self.logger.info(f"Best result was seen in epoch {self.best_epoch}")

    def do_sanity_check(self, sanity_check_dataloader):
        for i in range(self.args.epoch):
            self.logger.info(f"Epoch {i + 1}/{self.args.epoch}")
            deque(self.process_data(sanity_check_dataloader, True, i), maxlen=0)

    def do_evaluation(self, test_dataloader):
        deque(self.process_data(test_dataloader, False, 0), maxlen=0)
        self.logger.info(f"Accuracy: {self.last_metric_val * 100:.5f}%")
        self.logger.info(f"Loss: {self.last_loss:.5f}")
