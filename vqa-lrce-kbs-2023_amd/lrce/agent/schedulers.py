"""Learning-rate schedules of the reference agents (agent_base.py:46-72).

* ReduceLROnPlateau: torch's own (mode 'max', factor = lr_decay_factor, patience, min_lr), stepped with
  the validation metric (agent_base.py:161-162); it works on FusedAdamW unchanged because the
  optimizer re-reads its param_groups' lr every step.
* CosineAnnealingWarmupRestarts: the third-party package `cosine_annealing_warmup`
  (katsura-jp/pytorch-cosine-annealing-with-warmup, imported at agent_base.py:5; not vendored in the
  reference, not installed here).  Restated from its published algorithm: a linear warm-up from
  min_lr to max_lr over `warmup_steps`, then a half-cosine down to min_lr over the rest of the cycle;
  cycles restart with length (len - warmup) * cycle_mult + warmup and peak max_lr * gamma**cycle.
  The reference steps it with fractional epochs (agent_base.py:138: epoch + i / len(dl)) and passes
  warmup_steps = --lr-warm-up (a fraction of an epoch, args.py:36-41).
"""
import math

from torch.optim.lr_scheduler import ReduceLROnPlateau  # noqa: F401  (re-export, agent_base.py:64-71)


class CosineAnnealingWarmupRestarts:
    def __init__(self, optimizer, first_cycle_steps, cycle_mult=1.0, max_lr=0.1, min_lr=0.001, warmup_steps=0,
                 gamma=1.0, last_epoch=-1):
        if warmup_steps >= first_cycle_steps:
            raise ValueError("warmup_steps must be smaller than first_cycle_steps")
        self.optimizer = optimizer
        self.first_cycle_steps = first_cycle_steps
        self.cycle_mult = cycle_mult
        self.base_max_lr = max_lr
        self.max_lr = max_lr
        self.min_lr = min_lr
        self.warmup_steps = warmup_steps
        self.gamma = gamma
        self.cur_cycle_steps = first_cycle_steps
        self.cycle = 0
        self.step_in_cycle = last_epoch
        self.last_epoch = last_epoch
        # every group starts at min_lr (the package's init_lr)
        self.base_lrs = []
        for g in optimizer.param_groups:
            g["lr"] = min_lr
            self.base_lrs.append(min_lr)
        self.step()

    def get_lr(self):
        if self.step_in_cycle == -1:
            return list(self.base_lrs)
        if self.step_in_cycle < self.warmup_steps:
            return [(self.max_lr - b) * self.step_in_cycle / self.warmup_steps + b for b in self.base_lrs]
        span = self.cur_cycle_steps - self.warmup_steps
        phase = math.pi * (self.step_in_cycle - self.warmup_steps) / span
        return [b + (self.max_lr - b) * (1 + math.cos(phase)) / 2 for b in self.base_lrs]

    def step(self, epoch=None):
        if epoch is None:
            epoch = self.last_epoch + 1
            self.step_in_cycle += 1
            if self.step_in_cycle >= self.cur_cycle_steps:
                self.cycle += 1
                self.step_in_cycle -= self.cur_cycle_steps
                self.cur_cycle_steps = int((self.cur_cycle_steps - self.warmup_steps) * self.cycle_mult) + \
                    self.warmup_steps
        elif epoch >= self.first_cycle_steps:
            if self.cycle_mult == 1.0:
                self.step_in_cycle = epoch % self.first_cycle_steps
                self.cycle = int(epoch // self.first_cycle_steps)
            else:
                n = int(math.log(epoch / self.first_cycle_steps * (self.cycle_mult - 1) + 1, self.cycle_mult))
                self.cycle = n
                self.step_in_cycle = epoch - int(self.first_cycle_steps * (self.cycle_mult ** n - 1) /
                                                 (self.cycle_mult - 1))
                self.cur_cycle_steps = self.first_cycle_steps * self.cycle_mult ** n
        else:
            self.cur_cycle_steps = self.first_cycle_steps
            self.step_in_cycle = epoch
        self.max_lr = self.base_max_lr * self.gamma ** self.cycle
        self.last_epoch = math.floor(epoch)
        for g, lr in zip(self.optimizer.param_groups, self.get_lr()):
            g["lr"] = lr

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if k != "optimizer"}

    def load_state_dict(self, state):
        self.__dict__.update(state)
