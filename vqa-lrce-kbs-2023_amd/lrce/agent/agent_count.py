"""Repetition count (reference lrce/agent/agent_count.py): per-sample squared error (its mean is the
loss), the epoch metric is the mean squared error over all samples — lower is better — and step()
returns (loss, per-sample squared errors) like the reference."""
import torch.nn as nn

from .agent_base import AgentBase, get_logger


class AgentCount(AgentBase):
    METRIC = "MSE"
    HIGHER_IS_BETTER = False

    def __init__(self, model, gpu_id, args, log_enabled=True, is_eval=False, rank=None):
        super().__init__(model, gpu_id, args, log_enabled, is_eval, rank)
        self.logger = get_logger(__name__, self.rank)
        self.loss_func = nn.MSELoss(reduction="none")

    def task_loss(self, out, gt):
        return self.loss_func(out, gt.float())

    def pack_step(self, loss_value, out, gt, task_terms):
        return loss_value, task_terms

    def metric_terms(self, out, gt, task_terms):
        return task_terms.sum(), task_terms.numel()

    def unpack_step(self, result):
        loss, sq_err = result
        return loss, sq_err.sum().item(), sq_err.numel()
