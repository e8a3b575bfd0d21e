"""Learning-rate schedulers (reference: lr_scheduler.py:6-104).

``PolynomialDecayScheduler``: linear warmup over ``--warmup-updates`` (the
LR is exactly 0 at update 0, Q15), then
``(lr - end_lr) * (1 - (n - warmup) / (total - warmup)) ** power + end_lr``
and ``end_lr`` from ``--total-num-update`` on.  ``step(epoch)`` takes the
per-epoch base LR from the ``--lr`` list unless ``--force-anneal`` has been
reached.  State dict is ``{'best': ...}``.
"""
from __future__ import annotations


class _LRScheduler(object):
    def __init__(self, args, optimizer):
        self.args = args
        self.optimizer = optimizer
        self.best = None

    def state_dict(self):
        return {"best": self.best}

    def load_state_dict(self, state_dict):
        self.best = state_dict["best"]

    def step(self, epoch, val_loss=None):
        if val_loss is not None:
            self.best = val_loss if self.best is None else min(self.best, val_loss)

    def step_update(self, num_updates):
        return self.optimizer.get_lr()


class PolynomialDecayScheduler(_LRScheduler):
    def __init__(self, args, optimizer):
        super().__init__(args, optimizer)
        args.warmup_updates = getattr(args, "warmup_updates", 0) or 0
        self.lr = args.lr[0]
        self.warmup_factor = 1.0 / args.warmup_updates if args.warmup_updates > 0 else 1
        self.end_learning_rate = args.end_learning_rate
        self.total_num_update = args.total_num_update
        self.power = args.power
        self.optimizer.set_lr(self.warmup_factor * self.lr)

    def get_next_lr(self, epoch):
        lrs = self.args.lr
        if self.args.force_anneal is None or epoch < self.args.force_anneal:
            return lrs[min(epoch, len(lrs) - 1)]
        return self.optimizer.get_lr()

    def step(self, epoch, val_loss=None):
        super().step(epoch, val_loss)
        self.lr = self.get_next_lr(epoch)
        self.optimizer.set_lr(self.warmup_factor * self.lr)
        return self.optimizer.get_lr()

    def step_update(self, num_updates):
        w = self.args.warmup_updates
        if w > 0 and num_updates <= w:
            self.warmup_factor = num_updates / float(w)
            lr = self.warmup_factor * self.lr
        elif num_updates >= self.total_num_update:
            lr = self.end_learning_rate
        else:
            lr_range = self.lr - self.end_learning_rate
            pct_remaining = 1 - (num_updates - w) / (self.total_num_update - w)
            lr = lr_range * pct_remaining ** self.power + self.end_learning_rate
        self.optimizer.set_lr(lr)
        return self.optimizer.get_lr()


def build_lr_scheduler(args, optimizer):
    if args.lr_scheduler == "PolynomialDecayScheduler":
        return PolynomialDecayScheduler(args, optimizer)
    raise ValueError("unsupported lr_scheduler - {}".format(args.lr_scheduler))
