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


def polynomial_decay(n, base_lr, warmup, total, end_lr, power):
    """LR at update ``n`` after warmup: polynomial from ``base_lr`` (at ``warmup``) to ``end_lr`` (at ``total``)."""
    if n >= total:
        return end_lr
    frac_left = 1 - (n - warmup) / (total - warmup)
    return (base_lr - end_lr) * frac_left ** power + end_lr


class PolynomialDecayScheduler(_LRScheduler):
    """Warmup (from LR 0 at update 0) then polynomial decay; per-epoch base LR from ``--lr``."""

    def __init__(self, args, optimizer):
        super().__init__(args, optimizer)
        args.warmup_updates = getattr(args, "warmup_updates", 0) or 0
        self.lr = args.lr[0]
        self.end_learning_rate = args.end_learning_rate
        self.total_num_update = args.total_num_update
        self.power = args.power
        # scale of the base LR applied by step(epoch); only the warmup branch of step_update moves it
        self.warmup_factor = 1.0 / args.warmup_updates if args.warmup_updates > 0 else 1
        self.optimizer.set_lr(self.warmup_factor * self.lr)

    def get_next_lr(self, epoch):
        anneal_from = self.args.force_anneal
        if anneal_from is not None and epoch >= anneal_from:
            return self.optimizer.get_lr()  # annealing: keep whatever the updates reached
        per_epoch = self.args.lr
        return per_epoch[epoch] if epoch < len(per_epoch) else per_epoch[-1]

    def step(self, epoch, val_loss=None):
        super().step(epoch, val_loss)
        self.lr = self.get_next_lr(epoch)
        self.optimizer.set_lr(self.warmup_factor * self.lr)
        return self.optimizer.get_lr()

    def step_update(self, num_updates):
        warmup = self.args.warmup_updates
        in_warmup = 0 < warmup and num_updates <= warmup
        if in_warmup:
            self.warmup_factor = num_updates / float(warmup)
        lr = self.warmup_factor * self.lr if in_warmup else polynomial_decay(
            num_updates, self.lr, warmup, self.total_num_update, self.end_learning_rate, self.power)
        self.optimizer.set_lr(lr)
        return self.optimizer.get_lr()


def build_lr_scheduler(args, optimizer):
    if args.lr_scheduler == "PolynomialDecayScheduler":
        return PolynomialDecayScheduler(args, optimizer)
    raise ValueError("unsupported lr_scheduler - {}".format(args.lr_scheduler))
