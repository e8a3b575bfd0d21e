"""Training driver and launcher (reference: train.py:22-243).

Launch modes (reference: train.py:213-239), unchanged:
  (a) --distributed-init-method + --distributed-gpus > 1: spawn one process
      per local GPU with global rank = --distributed-rank + i (heterogeneous
      nodes contribute different --distributed-gpus);
  (b) init method with 1 GPU (or --distributed-no-spawn): run in-process;
  (c) no init method, world_size > 1: tcp://127.0.0.1:<random port>, spawn;
  (d) single process.
Additions: torchrun / env:// launches (RANK/LOCAL_RANK/WORLD_SIZE in the
environment) are detected; local index -> device uses --device-id-offset
(two launches sharing one node, Q24); CPU runs use gloo.

The epoch loop, stop criteria (lr > min_lr, max_epoch, max_update), update
grouping (--update-freq) and the per-update stats line are the reference's;
``--save-interval-updates`` additionally checkpoints mid-epoch (Q07).
"""
from __future__ import annotations

import collections
import math
import os
import random

import numpy as np
import torch

from hetseq_amd import checkpoint_utils, options, progress_bar, tasks, utils
from hetseq_amd.controller import Controller
from hetseq_amd.data import iterators
from hetseq_amd.meters import AverageMeter, StopwatchMeter
from hetseq_amd.parallel import distributed_utils
from hetseq_amd.runtime import profiling


def enable_deterministic(args):
    """Bitwise-reproducible training: must run before the process group is created."""
    import os

    os.environ.setdefault("NCCL_ALGO", "Ring")      # fixed RCCL reduction order
    os.environ.setdefault("NCCL_PROTO", "Simple")
    torch.use_deterministic_algorithms(True, warn_only=True)
    args.gemm_tuning = False  # tuned library solutions may split K with atomics


def main(args, init_distributed=False):
    assert args.max_tokens is not None or args.max_sentences is not None, \
        "Must specify batch size either with --max-tokens or --max-sentences"
    if torch.cuda.is_available() and not args.cpu:
        torch.cuda.set_device(args.device_id)
        from hetseq_amd.runtime import streams

        streams.reserve(torch.device("cuda", args.device_id))  # hardware queues before RCCL's streams
    if getattr(args, "profile", False):
        profiling.enable(True)
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    if getattr(args, "deterministic", False):
        enable_deterministic(args)
    if init_distributed:
        args.distributed_rank = distributed_utils.distributed_init(args)
    if distributed_utils.is_master(args):
        checkpoint_utils.verify_checkpoint_directory(args.save_dir)
    print(args, flush=True)

    task = tasks.setup_task(args)
    for valid_sub_split in args.valid_subset.split(","):
        task.load_dataset(valid_sub_split, combine=False, epoch=0)
    model = task.build_model(args)
    print("| num. model params: {} (num. trained: {})".format(
        sum(p.numel() for p in model.parameters()), sum(p.numel() for p in model.parameters() if p.requires_grad)))

    from hetseq_amd.runtime import gemm_tuning

    gemm_tuning.configure(args)  # process-global library-GEMM table: an entry-point decision
    controller = Controller(args, task, model)
    print("| training on {} GPUs".format(args.distributed_world_size))
    print("| max tokens per GPU = {} and max sentences per GPU = {}".format(args.max_tokens, args.max_sentences))

    extra_state, epoch_itr = checkpoint_utils.load_checkpoint(args, controller)
    if hasattr(task, "prepare_model_for_data"):
        task.prepare_model_for_data(controller.get_model(), args.train_subset)

    max_epoch = args.max_epoch or math.inf
    max_update = args.max_update or math.inf
    lr = controller.get_lr()
    train_meter = StopwatchMeter()
    train_meter.start()
    while (lr > args.min_lr
           and (epoch_itr.epoch < max_epoch or (epoch_itr.epoch == max_epoch and epoch_itr.resuming))
           and controller.get_num_updates() < max_update):
        train(args, controller, task, epoch_itr)
        valid_losses = [None]
        lr = controller.lr_step(epoch_itr.epoch, valid_losses[0])
        if epoch_itr.epoch % args.save_interval == 0:
            checkpoint_utils.save_checkpoint(args, controller, epoch_itr, valid_losses[0])
        reload_dataset = ":" in (getattr(args, "data", "") or "")
        epoch_itr = controller.get_train_iterator(epoch_itr.epoch, load_dataset=reload_dataset)
    train_meter.stop()
    from hetseq_amd.ops import bert_ops

    if controller.cuda:
        bert_ops.check_device_errors()
    print("| done training in {:.1f} seconds".format(train_meter.sum))
    if init_distributed:
        distributed_utils.shutdown(controller)
    return controller


def train(args, controller, task, epoch_itr):
    """Train the model for one epoch."""
    update_freq = args.update_freq[epoch_itr.epoch - 1] \
        if epoch_itr.epoch <= len(args.update_freq) else args.update_freq[-1]
    itr = epoch_itr.next_epoch_itr(fix_batches_to_gpus=args.fix_batches_to_gpus,
                                   shuffle=(epoch_itr.epoch >= args.curriculum))
    itr = iterators.GroupedIterator(itr, update_freq)
    progress = progress_bar.build_progress_bar(args, itr, epoch_itr.epoch, no_progress_bar="simple")
    extra_meters = collections.defaultdict(lambda: AverageMeter())
    max_update = args.max_update or math.inf
    for i, samples in enumerate(progress, start=epoch_itr.iterations_in_epoch):
        log_output = controller.train_step(samples)
        if log_output is None:
            continue
        stats = get_training_stats(controller)
        for k, v in log_output.items():
            if k in ["loss", "nll_loss", "ntokens", "nsentences", "sample_size"]:
                continue
            if "loss" in k or k == "accuracy":
                extra_meters[k].update(v, log_output["sample_size"])
            else:
                extra_meters[k].update(v)
            stats[k] = extra_meters[k].avg
        progress.log(stats, tag="train", step=stats["num_updates"])
        if i == 0:
            controller.get_meter("wps").reset()
            controller.get_meter("ups").reset()
        num_updates = controller.get_num_updates()
        if (args.save_interval_updates > 0 and num_updates % args.save_interval_updates == 0 and num_updates > 0):
            checkpoint_utils.save_checkpoint(args, controller, epoch_itr, None, end_of_epoch=False)
        if num_updates >= max_update:
            break


def get_training_stats(controller):
    stats = collections.OrderedDict()
    stats["loss"] = controller.get_meter("train_loss")
    if controller.get_meter("train_nll_loss").count > 0:
        nll_loss = controller.get_meter("train_nll_loss")
        stats["nll_loss"] = nll_loss
    else:
        nll_loss = controller.get_meter("train_loss")
    stats["ppl"] = _LazyPPL(nll_loss)
    stats["wps"] = controller.get_meter("wps")
    stats["ups"] = controller.get_meter("ups")
    stats["wpb"] = controller.get_meter("wpb")
    stats["bsz"] = controller.get_meter("bsz")
    stats["num_updates"] = controller.get_num_updates()
    stats["lr"] = controller.get_lr()
    stats["gnorm"] = controller.get_meter("gnorm")
    stats["clip"] = controller.get_meter("clip")
    stats["oom"] = controller.get_meter("oom")
    if controller.get_meter("loss_scale") is not None:
        stats["loss_scale"] = controller.get_meter("loss_scale")
    stats["wall"] = round(controller.get_meter("wall").elapsed_time)
    stats["train_wall"] = controller.get_meter("train_wall")
    return stats


class _LazyPPL(object):
    """ppl = 2 ** loss, evaluated only when printed (no per-step host sync)."""

    def __init__(self, meter):
        self.meter = meter

    def __str__(self):
        return "{:g}".format(utils.get_perplexity(self.meter.avg))

    def __format__(self, spec):
        return str(self)

    def __float__(self):
        return float(utils.get_perplexity(self.meter.avg))


def distributed_main(i, args, start_rank=0):
    args.device_id = distributed_utils.local_device_id(args, i)
    if args.distributed_rank is None:
        args.distributed_rank = start_rank + i
    return main(args, init_distributed=True)


def cli_main(argv=None):
    args = options.parse_cli(argv)
    env = distributed_utils.env_rank_info()
    if env is not None and args.distributed_init_method is None and env[2] > 1:
        # torchrun-style launch: one process per GPU already exists
        rank, local_rank, world = env
        args.distributed_init_method = "env://"
        args.distributed_world_size = world
        args.distributed_rank = rank
        args.device_id = distributed_utils.local_device_id(args, local_rank)
        return main(args, init_distributed=True)
    if args.distributed_init_method is not None:
        if args.distributed_gpus > 1 and not args.distributed_no_spawn:
            if torch.cuda.device_count() and not args.cpu:
                assert args.distributed_gpus + args.device_id_offset <= torch.cuda.device_count()
            start_rank = args.distributed_rank
            args.distributed_rank = None
            torch.multiprocessing.spawn(fn=distributed_main, args=(args, start_rank), nprocs=args.distributed_gpus)
        else:
            return distributed_main(args.device_id, args)
    elif args.distributed_world_size > 1:
        if torch.cuda.device_count() and not args.cpu:
            assert args.distributed_world_size <= torch.cuda.device_count()
        port = random.randint(10000, 20000)
        args.distributed_init_method = "tcp://127.0.0.1:{port}".format(port=port)
        args.distributed_rank = None
        torch.multiprocessing.spawn(fn=distributed_main, args=(args,), nprocs=args.distributed_world_size)
    else:
        return main(args)


if __name__ == "__main__":
    cli_main()
