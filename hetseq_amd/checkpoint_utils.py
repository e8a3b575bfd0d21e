"""Checkpoint save / resume (reference: checkpoint_utils.py:14-221).

File format (compatible both ways with the reference): a ``torch.save`` of
``{'args': Namespace, 'model': state_dict (tied decoder key duplicated),
'optimizer_history': [{'optimizer_name', 'lr_scheduler_state',
'num_updates'}], 'extra_state': {...}, 'last_optimizer_state': torch.optim
state_dict (CPU fp32)}``.

Fixes relative to the reference:
* Q01 -- ``extra_state`` is actually written (train iterator position, val
  loss, best, meters) so resume works; an empty ``extra_state`` (reference
  checkpoints) loads as "start of the recorded epoch".
* Q07 -- ``--save-interval-updates`` saves mid-epoch ``checkpoint_E_U.pt``.
* Q28 -- loading uses ``weights_only=True`` with ``argparse.Namespace``
  allow-listed (torch >= 2.6 default), never unpickling arbitrary objects.
* writes go to a temp file and are renamed atomically (3 attempts like the
  reference's ``torch_persistent_save``).
"""
from __future__ import annotations

import argparse
import collections
import logging
import os
import re
import shutil
import traceback
from collections import OrderedDict

import torch

from hetseq_amd import meters as meters_mod
from hetseq_amd.parallel import distributed_utils


def _checkpoint_names(args, epoch, updates, end_of_epoch, val_loss, improved):
    """File names this save writes, in priority order (the first is written, the rest copied)."""
    names = []
    if end_of_epoch and not args.no_epoch_checkpoints and epoch % args.save_interval == 0:
        names.append("checkpoint%d.pt" % epoch)
    if not end_of_epoch and args.save_interval_updates > 0 and updates % args.save_interval_updates == 0:
        names.append("checkpoint_%d_%d.pt" % (epoch, updates))
    if val_loss is not None and improved:
        names.append("checkpoint_best.pt")
    if not args.no_last_checkpoints:
        names.append("checkpoint_last.pt")
    return names


def _prune(save_dir, pattern, keep):
    """Delete all but the ``keep`` newest checkpoints whose names match ``pattern``."""
    for stale in checkpoint_paths(save_dir, pattern=pattern)[keep:]:
        if os.path.lexists(stale):
            os.remove(stale)


def save_checkpoint(args, controller, epoch_itr, val_loss, end_of_epoch=None):
    """Master-only save of the training state (reference: checkpoint_utils.py:14-83, with Q01/Q07 fixed)."""
    higher = args.maximize_best_checkpoint_metric
    prev_best = getattr(save_checkpoint, "best", val_loss)
    if val_loss is not None:
        save_checkpoint.best = max(val_loss, prev_best) if higher else min(val_loss, prev_best)
    if args.no_save:
        return
    controller.consolidate_optimizer()  # (every rank: the sharded optimizer's collective gather)
    if not distributed_utils.is_master(args):
        return
    clock = meters_mod.StopwatchMeter()
    clock.start()
    epoch, updates = epoch_itr.epoch, controller.get_num_updates()
    if end_of_epoch is None:
        end_of_epoch = epoch_itr.end_of_epoch()
    best = getattr(save_checkpoint, "best", None)
    improved = val_loss is not None and (not hasattr(save_checkpoint, "best") or (
        val_loss >= best if higher else val_loss <= best))
    extra_state = {"train_iterator": epoch_itr.state_dict(), "val_loss": val_loss}
    if hasattr(save_checkpoint, "best"):
        extra_state["best"] = save_checkpoint.best
    paths = [os.path.join(args.save_dir, n) for n in
             _checkpoint_names(args, epoch, updates, end_of_epoch, val_loss, improved)]
    if paths:
        controller.save_checkpoint(paths[0], extra_state)
        for dup in paths[1:]:
            shutil.copyfile(paths[0], dup)
        clock.stop()
        print("| saved checkpoint {} (epoch {} @ {} updates) (writing took {} seconds)".format(
            paths[0], epoch, updates, clock.sum))
    if not end_of_epoch and args.keep_interval_updates > 0:
        _prune(args.save_dir, r"checkpoint_\d+_(\d+)\.pt", args.keep_interval_updates)
    if args.keep_last_epochs > 0:
        _prune(args.save_dir, r"checkpoint(\d+)\.pt", args.keep_last_epochs)


def load_checkpoint(args, controller):
    """Load a checkpoint (if any) and restore the training iterator."""
    if args.distributed_rank == 0:
        os.makedirs(args.save_dir, exist_ok=True)
    if args.restore_file in ("checkpoint_last.pt", "checkpoint_best.pt"):
        checkpoint_path = os.path.join(args.save_dir, args.restore_file)
    else:
        checkpoint_path = args.restore_file
    import ast

    overrides = ast.literal_eval(args.optimizer_overrides) if isinstance(args.optimizer_overrides, str) \
        else args.optimizer_overrides
    extra_state = controller.load_checkpoint(checkpoint_path, args.reset_optimizer, args.reset_lr_scheduler,
                                             overrides, reset_meters=args.reset_meters)
    if extra_state is not None and "best" in extra_state and not args.reset_optimizer and not args.reset_meters:
        save_checkpoint.best = extra_state["best"]
    if extra_state is not None and not args.reset_dataloader:
        itr_state = extra_state.get("train_iterator")
        if itr_state is None:
            # reference-format checkpoints carry extra_state == {} (reference checkpoint_utils.py:204,
            # SURVEY Q01): rebuild the position the reference meant to save (its :50-55) from the
            # update count in optimizer_history and this run's batches per epoch
            epoch_itr = controller.get_train_iterator(epoch=0, load_dataset=True)
            per_rank = -(-len(epoch_itr) // max(1, epoch_itr.num_shards))
            # (the history's count, not the controller's: --reset-optimizer restarts the latter at 0)
            itr_state = iterator_state_from_updates(controller.checkpoint_num_updates(), per_rank, args.update_freq)
        else:
            epoch_itr = controller.get_train_iterator(epoch=itr_state["epoch"], load_dataset=True)
        epoch_itr.load_state_dict(itr_state)
    else:
        epoch_itr = controller.get_train_iterator(epoch=0, load_dataset=True)
    controller.lr_step(epoch_itr.epoch)
    return extra_state, epoch_itr


def iterator_state_from_updates(num_updates, batches_per_epoch, update_freq):
    """Iterator position after ``num_updates`` updates of ``batches_per_epoch`` micro-batches per
    epoch and rank, grouped by the per-epoch ``update_freq`` list (the last entry repeats), as the
    reference's ``EpochBatchIterator.state_dict`` would have recorded it: a finished epoch E gives
    ``{'epoch': E, 'iterations_in_epoch': 0}`` (the next run starts epoch E+1), a mid-epoch save
    the micro-batches consumed so far."""
    update_freq = list(update_freq) if isinstance(update_freq, (list, tuple)) else [int(update_freq)]
    epoch, left = 0, int(num_updates)
    while left > 0 and batches_per_epoch > 0:
        uf = update_freq[min(epoch, len(update_freq) - 1)]
        per_epoch = -(-batches_per_epoch // uf)
        if left < per_epoch:
            return {"epoch": epoch + 1, "iterations_in_epoch": left * uf}
        left -= per_epoch
        epoch += 1
    return {"epoch": epoch, "iterations_in_epoch": 0}


_SAFE = [argparse.Namespace, OrderedDict, collections.defaultdict]


def load_checkpoint_to_cpu(path, arg_overrides=None):
    with torch.serialization.safe_globals(_SAFE + _meter_classes()):
        state = torch.load(path, map_location="cpu", weights_only=True)
    args = state.get("args")
    if arg_overrides is not None and args is not None:
        for k, v in arg_overrides.items():
            setattr(args, k, v)
    return state


def _meter_classes():
    return [meters_mod.AverageMeter, meters_mod.TimeMeter, meters_mod.StopwatchMeter]


def checkpoint_paths(path, pattern=r"checkpoint(\d+)\.pt"):
    """Files in ``path`` fully matching ``pattern``, newest first by the captured number
    (by directory position when the pattern captures nothing)."""
    rx = re.compile(pattern)
    found = [(pos, rx.fullmatch(name)) for pos, name in enumerate(os.listdir(path))]
    keyed = sorted(((int(m.group(1)) if m.groups() else pos, m.group(0)) for pos, m in found if m), reverse=True)
    return [os.path.join(path, name) for _, name in keyed]


def torch_persistent_save(obj, filename):
    for i in range(3):
        try:
            tmp = filename + ".tmp"
            torch.save(obj, tmp)
            os.replace(tmp, filename)
            return
        except Exception:
            if i == 2:
                logging.error(traceback.format_exc())


def convert_state_dict_type(state_dict, ttype=torch.float32):
    if isinstance(state_dict, dict):
        out = OrderedDict()
        for k, v in state_dict.items():
            out[k] = convert_state_dict_type(v, ttype)
        return out
    if isinstance(state_dict, list):
        return [convert_state_dict_type(v, ttype) for v in state_dict]
    if torch.is_tensor(state_dict):
        t = state_dict.detach().to("cpu")
        return t.to(ttype) if t.is_floating_point() else t.clone()
    return state_dict


def _meters_state(meters):
    out = OrderedDict()
    for k, m in meters.items():
        if isinstance(m, meters_mod.AverageMeter):
            out[k] = {"type": "avg", **m.state_dict()}
        elif isinstance(m, meters_mod.StopwatchMeter):
            out[k] = {"type": "stopwatch", "sum": m.sum, "n": m.n}
        elif isinstance(m, meters_mod.TimeMeter):
            out[k] = {"type": "time", "n": m.n, "elapsed": m.elapsed_time}
    return out


def restore_meters(meters, state):
    for k, st in state.items():
        if k not in meters or not isinstance(st, dict):
            continue
        m = meters[k]
        if st.get("type") == "avg" and isinstance(m, meters_mod.AverageMeter):
            m.load_state_dict(st)
        elif st.get("type") == "stopwatch" and isinstance(m, meters_mod.StopwatchMeter):
            m.sum, m.n = st["sum"], st["n"]
        elif st.get("type") == "time" and isinstance(m, meters_mod.TimeMeter):
            m.reset(init=st["elapsed"])
            m.n = st["n"]


def save_state(filename, args, model_state_dict, criterion, optimizer, lr_scheduler, num_updates, optim_history=None,
               extra_state=None):
    if optim_history is None:
        optim_history = []
    if extra_state is None:
        extra_state = {}
    extra = dict(extra_state)
    if "train_meters" in extra:
        extra["train_meters"] = _meters_state(extra["train_meters"])
    state_dict = {
        "args": args,
        "model": convert_state_dict_type(model_state_dict) if model_state_dict else {},
        "optimizer_history": optim_history + [{
            "optimizer_name": optimizer.__class__.__name__,
            "lr_scheduler_state": lr_scheduler.state_dict(),
            "num_updates": num_updates,
        }],
        "extra_state": extra,
    }
    if not args.no_save_optimizer_state:
        state_dict["last_optimizer_state"] = convert_state_dict_type(optimizer.state_dict())
    torch_persistent_save(state_dict, filename)


def verify_checkpoint_directory(save_dir):
    """Create ``save_dir`` if needed and prove it is writable (fails early, before training)."""
    os.makedirs(save_dir, exist_ok=True)
    probe = os.path.join(save_dir, "dummy")
    try:
        open(probe, "w").close()
    except OSError:
        print("| Unable to access checkpoint save directory: {}".format(save_dir))
        raise
    os.remove(probe)
