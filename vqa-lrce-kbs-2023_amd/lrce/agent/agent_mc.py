"""Multiple-choice agent (reference lrce/agent/agent_mc.py): cross-entropy over the 5 choices, or
with --use-hinge-loss the multi-class hinge loss of agent_mc.py:20-41 (a per-sample Python loop
there, one vectorised expression here — same value and gradient)."""
import torch

from .agent_base import AgentBase, get_logger


def hinge_loss(out, gt, margin):
    """mean_i sum_{j != gt_i} max(0, out[i, j] - out[i, gt_i] + margin)   (agent_mc.py:20-41)."""
    out = out.float()
    correct = out.gather(1, gt.view(-1, 1))
    terms = torch.clamp(out - correct + margin, min=0.0)
    keep = torch.ones_like(terms).scatter_(1, gt.view(-1, 1), 0.0)
    return (terms * keep).sum(dim=1).mean()


class AgentMC(AgentBase):
    def __init__(self, model, gpu_id, args, log_enabled=True, is_eval=False):
        super().__init__(model, gpu_id, args, log_enabled, is_eval)
        if getattr(self.args, "use_hinge_loss", False):
            self.loss_func = self.hinge_loss
        self.logger = get_logger(__name__, gpu_id)

    def hinge_loss(self, out, gt):
        return hinge_loss(out, gt, self.args.margin)

    def step(self, video_clips, texts, texts_attention_mask, texts_type_ids, ground_truth, is_train):
        out = self._forward(video_clips, texts, texts_attention_mask, texts_type_ids)
        gt = ground_truth.to(self.device)
        task_loss = self.loss_func(out.float(), gt)
        loss = self._regularised(task_loss)
        if is_train:
            self._backward_and_update(task_loss)
        prediction = torch.argmax(out, dim=1)
        total_data = prediction.shape[0]
        total_correct = torch.sum(prediction == gt).item()
        return loss.item(), total_correct, total_data
