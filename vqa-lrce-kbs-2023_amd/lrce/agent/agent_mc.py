"""Multiple choice (reference lrce/agent/agent_mc.py): cross-entropy over the choices, or with
--use-hinge-loss the multi-class hinge loss of agent_mc.py:20-41 — a per-sample Python loop there,
one vectorised expression here (same value and gradient, tests/test_agent_cpu.py)."""
import torch

from .agent_base import AgentBase, get_logger


def hinge_loss(out, gt, margin):
    """mean_i sum_{j != gt_i} max(0, out[i, j] - out[i, gt_i] + margin)."""
    out = out.float()
    margins = torch.clamp(out - out.gather(1, gt.view(-1, 1)) + margin, min=0.0)
    others = torch.ones_like(margins).scatter_(1, gt.view(-1, 1), 0.0)
    return (margins * others).sum(dim=1).mean()


class AgentMC(AgentBase):
    def __init__(self, model, gpu_id, args, log_enabled=True, is_eval=False, rank=None):
        super().__init__(model, gpu_id, args, log_enabled, is_eval, rank)
        if getattr(self.args, "use_hinge_loss", False):
            self.loss_func = self.hinge_loss
        self.logger = get_logger(__name__, self.rank)

    def hinge_loss(self, out, gt):
        return hinge_loss(out, gt, self.args.margin)
