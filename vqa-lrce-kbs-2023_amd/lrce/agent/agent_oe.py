"""Open-ended QA agent (reference lrce/agent/agent_oe.py:19-48): cross-entropy over the answer
vocabulary (ignore_index -100) + reg * L2, top-1 accuracy."""
import torch

from .agent_base import AgentBase, get_logger


class AgentOE(AgentBase):
    def __init__(self, model, gpu_id, args, log_enabled=True, is_eval=False):
        super().__init__(model, gpu_id, args, log_enabled, is_eval)
        self.logger = get_logger(__name__, gpu_id)

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
