"""Repetition-count agent (reference lrce/agent/agent_count.py): MSE (reduction 'none', averaged for
the loss) + reg * L2; the tracked metric is the mean squared error, lower is better."""
import torch
import torch.nn as nn

from .agent_base import AgentBase, get_logger


class AgentCount(AgentBase):
    def __init__(self, model, gpu_id, args, log_enabled=True, is_eval=False):
        super().__init__(model, gpu_id, args, log_enabled, is_eval)
        self.logger = get_logger(__name__, gpu_id)
        self.loss_func = nn.MSELoss(reduction="none")

    def is_metric_val_better(self, epoch=None):
        if self.best_metric_val is None or self.last_metric_val < self.best_metric_val:
            self.best_metric_val = self.last_metric_val
            self.best_epoch = epoch
            return True
        return False

    def step(self, video_clips, texts, texts_attention_mask, texts_type_ids, ground_truth, is_train):
        out = self._forward(video_clips, texts, texts_attention_mask, texts_type_ids)
        mse_loss = self.loss_func(out.float(), ground_truth.to(self.device).float())
        task_loss = torch.mean(mse_loss)
        loss = self._regularised(task_loss)
        if is_train:
            self._backward_and_update(task_loss)
        return loss.item(), mse_loss.detach()

    def process_data(self, dl, is_train, epoch):
        """agent_count.py:54-116: the accumulated metric is sum(mse) / count over the ranks."""
        if is_train:
            self.logger.info("Training Phase")
        elif not self.is_eval:
            self.logger.info("Validation Phase")
        mse_counter = torch.zeros(2, device=self.device)
        batch_losses = torch.zeros(len(dl), device=self.device)
        avg_losses, avg_mse = float("nan"), float("nan")
        for i, batch_data in enumerate(dl):
            if not is_train:
                self.model.eval()
                with torch.no_grad():
                    b_loss, mse_loss = self.step(*batch_data, is_train=False)
            else:
                self.model.train()
                b_loss, mse_loss = self.step(*batch_data, is_train=True)
                self.counter += 1
                if getattr(self.args, "use_cosine_scheduler", False):
                    self.scheduler.step(epoch + i / len(dl))
                for k in range(len(self.optim.param_groups)):
                    self.write_summary(f"LR Scheduler/{k}", self.optim.param_groups[k]["lr"], self.counter)
                self.write_summary("Training/Batch Loss", b_loss, self.counter)
                self.write_summary("Training/Batch MSE", torch.mean(mse_loss).item(), self.counter)
                yield i
            if self.gpu_id != 0:
                mse_counter.zero_()
            mse_counter[0] += torch.sum(mse_loss).item()
            mse_counter[1] += len(mse_loss)
            batch_losses[i] = b_loss
            self._reduce(mse_counter)
            nz = batch_losses[batch_losses.nonzero()]
            avg_losses = nz.mean().item() if nz.numel() else 0.0
            avg_mse = (mse_counter[0] / mse_counter[1]).item()
        if not is_train:
            self.last_loss = avg_losses
            self.last_metric_val = avg_mse
            if not self.is_eval and not getattr(self.args, "use_cosine_scheduler", False):
                self.scheduler.step(-avg_mse)
            self.write_summary("Validation/Loss", avg_losses, epoch)
            self.write_summary("Validation/MSE", avg_mse, epoch)
        else:
            self.write_summary("Training/Loss", avg_losses, epoch)
            self.write_summary("Training/MSE", avg_mse, epoch)
        yield -1
