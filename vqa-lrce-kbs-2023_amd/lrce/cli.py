"""Command-line surface of the reference scripts (args.py:5-155 for train.py / eval.py, parser.py:5-114
for train_ddp.py) and the drivers they run (train_ddp.py:16-131, eval.py:16-95).

Flags, defaults and post-processing are the reference's: the per-dataset model config is merged over
the parsed flags (configs/<dataset>.json — restated below as CONFIGS, including msrvtt's
"msvrvtt-qa-oe" dataset string, which the merge copies into args.dataset), a single --lr is expanded
to the three parameter groups, an empty --temporal-scale falls back to the default, and the
scheduler / hinge flags that do not apply are deleted from the namespace.  The only difference in
the defaults is that train.py (args.py) uses temporal scale [1, 2, 3] and train_ddp.py (parser.py)
uses [3].

Additive flags (absent from the reference, no effect on its flags):
  --synthetic N        train/eval on N synthetic items with the reference item contract
                       (lrce/dataset/synthetic.py) instead of decoded videos; --dataset-dir is then
                       not needed.  Video decoding and tokenisation are out of scope for this build.
  --synthetic-val N    size of the synthetic validation / test split (default max(N // 4, batch)).
  --seed S             synthetic data seed.
  --allow-random-init  train although the Swin checkpoint / local BERT weights are missing (the
                       reference asserts the checkpoint, e2e.py:11); implied by --synthetic.
Launch: under torchrun (RANK / WORLD_SIZE / LOCAL_RANK in the environment) each process is one rank
on device LOCAL_RANK; otherwise one process per visible GPU is spawned, as the reference's mp.spawn
does.  The process group is "nccl" (RCCL over xGMI) with MASTER_ADDR 127.0.0.1.
"""
import argparse
import copy
import os
import sys

DATASETS = ["msvd-qa-oe", "msrvtt-qa-oe", "tgif-frameqa", "tgif-count", "tgif-action", "tgif-transition"]

_BASE = {"feature_dim": 768, "frame_sample_size": 5, "video_feature_res": [7, 7], "video_feature_dim": 1024}
CONFIGS = {   # configs/*.json
    "msrvtt-qa-oe": dict(_BASE, dataset="msvrvtt-qa-oe", text_seq_len=37, task_type="oe", num_classes=1500),
    "msvd-qa-oe": dict(_BASE, dataset="msvd-qa-oe", text_seq_len=32, task_type="oe", num_classes=1000),
    "tgif-action": dict(_BASE, dataset="tgif-action", text_seq_len=40, task_type="mc", num_classes=1),
    "tgif-count": dict(_BASE, dataset="tgif-count", text_seq_len=30, task_type="count", num_classes=1),
    "tgif-frameqa": dict(_BASE, dataset="tgif-frameqa", text_seq_len=30, task_type="oe", num_classes=1000),
    "tgif-transition": dict(_BASE, dataset="tgif-transition", text_seq_len=40, task_type="mc", num_classes=1),
}


def _additive(p):
    p.add_argument("--synthetic", type=int, default=0, help="use N synthetic items (no video decoding)")
    p.add_argument("--synthetic-val", type=int, default=0, help="synthetic validation/test items")
    p.add_argument("--seed", type=int, default=0, help="synthetic data seed")
    p.add_argument("--allow-random-init", action="store_true",
                   help="train from random backbones when the pretrained Swin / BERT weights are missing")
    p.add_argument("--eager", action="store_true",
                   help="launch every training step from Python instead of replaying it from HIP graphs")
    p.add_argument("--log-interval", type=int, default=50,
                   help="steps between reads of the device-side loss / metric sums")
    p.add_argument("--grad-reduce-dtype", choices=["bf16", "f32"], default="bf16",
                   help="data-parallel gradient exchange: bf16 on the wire with the cross-rank sum in f32 "
                        "(default), or f32 all-reduce")


def _merge_config(result):
    vars(result).update(copy.deepcopy(CONFIGS[result.dataset]))


def _check_data(p, result):
    if not result.synthetic and not result.dataset_dir:
        p.error("the following arguments are required: --dataset-dir (or --synthetic N)")


def parse_arg_train(argv=None, temporal_default=(3,)):
    """parser.py:parse_arg_train (train_ddp.py); temporal_default=(1, 2, 3) gives args.py's (train.py)."""
    p = argparse.ArgumentParser(description="Train Model")
    p.add_argument("--dataset", help="Dataset to use", choices=DATASETS, type=str, required=True)
    p.add_argument("--dataset-dir", help="Directory path to dataset for train and validation")
    p.add_argument("--log-dir", help="Log directory", default="./runs")
    p.add_argument("--ckpt-interval", help="How many epoch between checkpoints", default=1, type=int)
    p.add_argument("--model-path", help="Load pretrained model")
    p.add_argument("--batch-size", help="Batch size for training", default=20, type=int)
    p.add_argument("--eval-per-epoch", help="Total validation per epoch", default=1, type=int)
    p.add_argument("--epoch", help="Total epoch", default=20, type=int)
    p.add_argument("--drop-out-rate", help="Drop out rate for training", default=0.5, type=float)
    p.add_argument("--lr", help="Learning rate for training", nargs="+", default=[5e-6], type=float)
    p.add_argument("--min-lr", help="Minimum learning rate after decaying", default=1e-8, type=float)
    p.add_argument("--temporal-scale", help="Scales for multisegment sampling", nargs="+",
                   default=list(temporal_default), type=int)
    # the reference declares type=int with a float default 0.5 (argparse does not convert defaults)
    p.add_argument("--patience", help="Number of stagnant epoch before decay (only for reduce on plateau "
                   "scheduler)", default=0.5, type=int)
    p.add_argument("--lr-decay-factor", help="Learning rate decay factor (after full-cycle for cosine scheduler)",
                   default=0.5, type=float)
    p.add_argument("--lr-warm-up", help="Percentage of epoch to do linear warmup [0,1)", default=0.1, type=float)
    p.add_argument("--lr-restart-epoch", help="Number of epoch before restarting the learning rate (only for "
                   "cosine annealing scheduler)", default=2, type=int)
    p.add_argument("--lr-restart-mul", help="Multiplier for lr-restart-epoch after restart (only for cosine "
                   "annealing scheduler)", default=1, type=int)
    p.add_argument("--use-cosine-scheduler", help="Whether to use cosine annealing scheduler or reduce on "
                   "plateau scheduler", action="store_true")
    p.add_argument("--reg-strength", help="Weight for L2 regularization", default=0.001, type=float)
    p.add_argument("--num-workers", help="Number of workers for dataloader", default=2, type=int)
    p.add_argument("--use-hinge-loss", help="Use hinge loss instead of cross entropy (for mc task)",
                   action="store_true")
    p.add_argument("--margin", help="Margin for hingle loss (only for mc task)", default=1, type=float)
    p.add_argument("--debug-mode", help="If on, it will not write logs and checkpoints", action="store_true")
    p.add_argument("--sanity-check", help="Sanity check by overfitting model with very small dataset",
                   action="store_true")
    p.add_argument("--comment", help="Additional comment if needed", default="", type=str)
    _additive(p)
    result = p.parse_args(argv)
    _check_data(p, result)
    if result.use_cosine_scheduler:
        del vars(result)["patience"]
    else:
        del vars(result)["lr_restart_epoch"]
        del vars(result)["lr_restart_mul"]
        del vars(result)["lr_warm_up"]
    if not result.use_hinge_loss:
        del vars(result)["margin"]
    if result.comment == "":
        del vars(result)["comment"]
    _merge_config(result)
    if len(result.lr) == 1:
        result.lr = result.lr * 3
    if len(result.temporal_scale) < 1:
        result.temporal_scale = list(temporal_default)
    return result


def parse_arg_eval(argv=None):
    """args.py:parse_arg_eval (eval.py)."""
    p = argparse.ArgumentParser(description="Train Model")
    p.add_argument("--dataset", help="Dataset to use", choices=DATASETS, type=str, required=True)
    p.add_argument("--dataset-dir", help="Directory path to dataset for train and validation")
    p.add_argument("--model-path", help="Load pretrained model", required=True)
    p.add_argument("--batch-size", help="Batch size for training", default=20, type=int)
    p.add_argument("--temporal-scale", help="Scales for multisegment sampling", nargs="+", default=[3], type=int)
    p.add_argument("--num-workers", help="Number of workers for dataloader", default=2, type=int)
    p.add_argument("--use-hinge-loss", help="Use hinge loss instead of cross entropy (for mc task)",
                   action="store_true")
    p.add_argument("--margin", help="Margin for hingle loss (only for mc task)", default=1, type=float)
    p.add_argument("--reg-strength", help="Weight for L2 regularization", default=0, type=float)
    _additive(p)
    result = p.parse_args(argv)
    _check_data(p, result)
    _merge_config(result)
    if len(result.temporal_scale) < 1:
        result.temporal_scale = [3]
    return result


# ---------------------------------------------------------------------------------------------- drivers
def factories(task_type):
    """train_ddp.py:78-90 / eval.py:55-67: model and agent classes per task type."""
    from .agent import AgentCount, AgentMC, AgentOE
    from .models.e2e import E2ECount, E2EMultipleChoice, E2EOpenEnded
    table = {"oe": (E2EOpenEnded, AgentOE), "mc": (E2EMultipleChoice, AgentMC), "count": (E2ECount, AgentCount)}
    if task_type not in table:
        raise SystemExit("Unsupported task type")
    return table[task_type]


def datasets(a, splits):
    """The reference builds E2EMicrosoftDataset / E2ETGIFDataset from annotation files and videos
    (train_ddp.py:24-75); this build serves the same item contract from SyntheticQADataset.  For
    eval.py (the only split is 'test') --synthetic N is the size of that split."""
    from .dataset import SyntheticQADataset
    if not a.synthetic:
        raise NotImplementedError("video/annotation readers are out of scope for this build (SURVEY §8 f); "
                                  "run with --synthetic N")
    held = a.synthetic_val or max(a.synthetic // 4, a.batch_size)
    sizes = {"train": a.synthetic, "val": held, "test": a.synthetic if list(splits) == ["test"] else held}
    out = []
    for i, s in enumerate(splits):
        out.append(SyntheticQADataset(sizes[s], task_type=a.task_type, max_text_token_len=a.text_seq_len,
                                      temporal_scale=a.temporal_scale, frames_per_clip=a.frame_sample_size,
                                      num_classes=a.num_classes, seed=a.seed * 10 + i))
    return out


def _loader(ds, a):
    import torch
    from torch.utils.data.distributed import DistributedSampler
    return torch.utils.data.DataLoader(ds, batch_size=a.batch_size, shuffle=False, num_workers=a.num_workers,
                                       pin_memory=True, sampler=DistributedSampler(ds))


def local_rank(rank):
    """Device index of this process: LOCAL_RANK under torchrun (multi-node safe), else the rank
    (mp.spawn on one node, train_ddp.py:17-18)."""
    return int(os.environ.get("LOCAL_RANK", rank))


def _setup(rank, world):
    """Process group over RCCL; the global rank joins the group, the local rank picks the device
    (train_ddp.py:10-13, 17-18)."""
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "12355")
    dev = local_rank(rank)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))
    return dev


def train_main(rank, world, a, val_split="test"):
    """train_ddp.py:16-131 (val_split 'test') / train.py (val_split 'val')."""
    import logging
    import torch.distributed as dist
    dev = _setup(rank, world)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")
    model_factory, agent_factory = factories(a.task_type)
    train_ds, val_ds = datasets(a, ["train", val_split])
    model = model_factory(a.feature_dim, a.num_classes, a.drop_out_rate, a.video_feature_res, a.video_feature_dim,
                          a.frame_sample_size, a.temporal_scale, a.text_seq_len)
    if not (model.pretrained_loaded or a.model_path or a.synthetic or a.allow_random_init):
        raise SystemExit("pretrained Swin (./pretrained_models/swin_base_patch244_window877_kinetics600_22k.pth) "
                         "and BERT (./pretrained_models/bert-base-uncased) weights are required for a real run "
                         "(reference e2e.py:11); pass --allow-random-init to train from random backbones")
    trainer = agent_factory(model, dev, a, not a.debug_mode and not a.sanity_check, rank=rank)
    if a.model_path:
        trainer.load_checkpoint(a.model_path)
    train_dl, val_dl = _loader(train_ds, a), _loader(val_ds, a)
    if a.sanity_check:
        trainer.do_sanity_check(train_dl)
    else:
        trainer.do_training(train_dl, val_dl, a.eval_per_epoch)
    dist.destroy_process_group()
    return trainer


def eval_main(rank, world, a):
    """eval.py:16-95."""
    import logging
    import torch.distributed as dist
    dev = _setup(rank, world)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")
    model_factory, agent_factory = factories(a.task_type)
    (test_ds,) = datasets(a, ["test"])
    model = model_factory(feature_dim=a.feature_dim, num_classes=a.num_classes, video_feature_res=a.video_feature_res,
                          video_feature_dim=a.video_feature_dim, frame_sample_size=a.frame_sample_size,
                          temporal_scale=a.temporal_scale, text_seq_len=a.text_seq_len)
    evaluator = agent_factory(model, dev, a, False, True, rank=rank)
    evaluator.load_checkpoint(a.model_path)
    evaluator.do_evaluation(_loader(test_ds, a))
    dist.destroy_process_group()
    return evaluator


def launch(fn, *fn_args):
    """torchrun: run this rank.  Plain `python script.py`: one spawned process per visible GPU."""
    if "WORLD_SIZE" in os.environ and "RANK" in os.environ:
        rank = int(os.environ["RANK"])
        fn(rank, int(os.environ["WORLD_SIZE"]), *fn_args)
        return
    import torch
    import torch.multiprocessing as mp
    world = torch.cuda.device_count()
    if world < 1:
        sys.exit("no HIP device visible: the LRCE native path runs on MI355X only")
    mp.spawn(fn, nprocs=world, args=(world, *fn_args))
