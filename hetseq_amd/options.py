"""Command-line flag system.

Flag-for-flag parity with the reference parser (reference: options.py:5-290,
SURVEY Appendix A): same names, aliases, defaults and task/optimizer
dependent groups, including the reference's odd spellings
(``--config_file``, ``--max_pred_length``, ``--num_file``, ``--adadelta_rho``,
``--dadelta_weight_decay``, ``--lr_scheduler``).  List flags (``--lr``,
``--update-freq``) accept the reference syntax ("0.1,0.05" or "[1, 2]") but
are parsed with ``ast.literal_eval`` instead of ``eval``.

MI355X/framework extensions live in their own argument group (they never
change a reference default):
  --dtype {fp32,bf16}       compute precision (fp32 = reference parity)
  --fused / --no-fused      use the gfx950 HIP kernel path when on GPU
  --device-id-offset N      map local rank i -> device i+N (heterogeneous launches on one node, Q24)
  --per-rank-seed           different dropout streams per rank (reference: identical, Q14)
  --check-consistency N     all-reduce a parameter checksum every N updates
  --collective-timeout S    timeout (seconds) for process-group collectives (and the RCCL watchdog)
  --comm-engine E           gradient collectives: native RCCL engine (auto on GPU+nccl) or c10d
  --shard-optimizer {auto,on,off}  data-parallel Adam sharded over the ranks (reduce-scatter / all-gather)
  --no-sparse-embedding-exchange  all-reduce the embedding tables densely in the last bucket
                            (default: early dense bucket + sparse row exchange, parallel/tied.py)
  --checkpoint-activations  recompute encoder layers in backward
  --json-log PATH           append one JSON object per logged update
  --profile                 roctx ranges + per-phase hipEvent timing
  --no-gemm-tuning          skip the measured GEMM selection table
  --deterministic           bitwise-reproducible mode (fixed RCCL algorithm, deterministic torch ops)
  --hip-graph               replay the captured update as one HIP graph (launch-bound configurations)
"""
from __future__ import annotations

import argparse
import ast

import torch


def _device_count():
    try:
        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


def get_training_parser(task="bert", optimizer="adam", lr_scheduler="PolynomialDecayScheduler"):
    parser = argparse.ArgumentParser(allow_abbrev=False)
    parser.add_argument("--no-progress-bar", action="store_true", help="disable progress bar")
    parser.add_argument("--seed", default=19940802, type=int, metavar="N", help="pseudo random number generator seed")
    parser.add_argument("--cpu", action="store_true", help="use CPU instead of the GPU")
    parser.add_argument("--log-interval", type=int, default=1, metavar="N",
                        help="log progress every N batches (when progress bar is disabled)")
    parser.add_argument("--log-format", default="simple", help="log format to use", choices=["none", "simple", "json"])

    add_dataset_args(parser, train=True, task=task)
    add_distributed_training_args(parser)
    add_optimization_args(parser, optimizer=optimizer, lr_scheduler=lr_scheduler)
    add_checkpoint_args(parser)
    add_mi355x_args(parser)
    return parser


def add_dataset_args(parser, train=False, gen=False, task="bert"):
    group = parser.add_argument_group("Dataset and data loading")
    group.add_argument("--num-workers", default=0, type=int, metavar="N",
                       help="how many subprocesses (or native reader threads) to use for data loading")
    group.add_argument("--max-tokens", type=int, metavar="N", help="maximum number of tokens in a batch")
    group.add_argument("--max-sentences", "--batch-size", type=int, metavar="N",
                       help="maximum number of sentences in a batch")
    group.add_argument("--required-batch-size-multiple", default=1, type=int, metavar="N",
                       help="batch size will be a multiplier of this value")
    if train:
        group.add_argument("--train-subset", default="train", metavar="SPLIT", choices=["train", "valid", "test"],
                           help="data subset to use for training (train, valid, test)")
        group.add_argument("--valid-subset", default="valid", metavar="SPLIT",
                           help="comma separated list of data subsets to use for validation")
        group.add_argument("--validate-interval", type=int, default=1, metavar="N", help="validate every N epochs")
        group.add_argument("--disable-validation", action="store_true", help="disable validation")
        group.add_argument("--max-tokens-valid", type=int, metavar="N",
                           help="maximum number of tokens in a validation batch (defaults to --max-tokens)")
        group.add_argument("--max-sentences-valid", type=int, metavar="N",
                           help="maximum number of sentences in a validation batch (defaults to --max-sentences)")
        group.add_argument("--curriculum", default=0, type=int, metavar="N",
                           help="don't shuffle batches for first N epochs")
        if task == "bert":
            parser.add_argument("--task", type=str, default="bert")
            parser.add_argument("--data", type=str, help="path including data")
            group.add_argument("--dict", type=str, metavar="PATH of a file", help="PATH to dictionary")
            group.add_argument("--config_file", type=str, metavar="PATH of a file",
                               help="PATH to bert model configuration", required=True)
            group.add_argument("--max_pred_length", type=int, default=512, help="max number of tokens in a sentence")
            group.add_argument("--num_file", type=int, default=0, help="number of file to run, 0 for all")
        elif task == "mnist":
            parser.add_argument("--task", type=str, default="mnist")
            parser.add_argument("--data", type=str, help="path including data")
        else:
            raise ValueError("unsupported task: {}".format(task))


def add_distributed_training_args(parser):
    group = parser.add_argument_group("Distributed training")
    group.add_argument("--distributed-world-size", type=int, metavar="N", default=max(1, _device_count()),
                       help="total number of GPUs across all nodes (default: all visible GPUs)")
    group.add_argument("--distributed-rank", default=0, type=int, help="rank of the current GPU")
    group.add_argument("--distributed-gpus", default=4, type=int,
                       help="number of gpus used in the current worker/node")
    group.add_argument("--distributed-backend", default="nccl", type=str,
                       help="distributed backend (nccl = RCCL on ROCm; gloo for CPU)")
    group.add_argument("--distributed-init-method", default=None, type=str,
                       help="typically tcp://hostname:port or file:///shared/path (env:// also accepted)")
    group.add_argument("--device-id", "--local_rank", default=0, type=int,
                       help="which GPU to use (usually configured automatically)")
    group.add_argument("--distributed-no-spawn", action="store_true",
                       help="do not spawn multiple processes even if multiple GPUs are visible")
    group.add_argument("--ddp-backend", default="c10d", type=str, choices=["c10d"],
                       help="DistributedDataParallel backend (kept for CLI parity; the flat-bucket engine is used)")
    group.add_argument("--bucket-cap-mb", default=25, type=int, metavar="MB", help="bucket size for reduction")
    group.add_argument("--fix-batches-to-gpus", action="store_true",
                       help="don't shuffle batches between GPUs; requires a dataset that supports prefetch")
    group.add_argument("--find-unused-parameters", default=False, action="store_true",
                       help="tolerate parameters that receive no gradient in a step")
    group.add_argument("--fast-stat-sync", default=False, action="store_true",
                       help="Enable fast sync of stats between nodes (one all-reduce of 6 doubles)")
    return group


def add_optimization_args(parser, optimizer="adam", lr_scheduler="PolynomialDecayScheduler"):
    group = parser.add_argument_group("Optimization")
    group.add_argument("--max-epoch", "--me", default=0, type=int, metavar="N",
                       help="force stop training at specified epoch")
    group.add_argument("--max-update", "--mu", default=0, type=int, metavar="N",
                       help="force stop training at specified update")
    group.add_argument("--clip-norm", default=25, type=float, metavar="NORM", help="clip threshold of gradients")
    group.add_argument("--update-freq", default="1", metavar="N1,N2,...,N_K",
                       type=lambda uf: eval_str_list(uf, type=int),
                       help="update parameters every N_i batches, when in epoch i")
    group.add_argument("--lr", "--learning-rate", default="0.25", type=eval_str_list, metavar="LR_1,LR_2,...,LR_N",
                       help="learning rate for the first N epochs; all epochs >N using LR_N")
    group.add_argument("--min-lr", default=-1, type=float, metavar="LR",
                       help="stop training when the learning rate reaches this minimum")
    group.add_argument("--use-bmuf", default=False, action="store_true",
                       help="block-momentum model averaging instead of per-step gradient all-reduce")
    if optimizer in ("adam", "lamb"):
        group.add_argument("--optimizer", default=optimizer, type=str, help="optimizer name")
        group.add_argument("--adam-betas", default="(0.9, 0.999)", metavar="B", help="betas for Adam optimizer")
        group.add_argument("--adam-eps", type=float, default=1e-8, metavar="D", help="epsilon for Adam optimizer")
        group.add_argument("--weight-decay", "--wd", default=0.0, type=float, metavar="WD", help="weight decay")
    elif optimizer == "adadelta":
        group.add_argument("--optimizer", default="adadelta", type=str, help="optimizer name")
        group.add_argument("--adadelta_rho", default="0.9", type=float)
        group.add_argument("--adadelta_eps", default="1e-6", type=float)
        group.add_argument("--dadelta_weight_decay", default="0", type=float)
    else:
        raise ValueError("unsupported optimizer: {}".format(optimizer))
    if lr_scheduler == "PolynomialDecayScheduler":
        group.add_argument("--lr_scheduler", default="PolynomialDecayScheduler", type=str,
                           help="learning-rate scheduler")
        group.add_argument("--force-anneal", "--fa", type=int, metavar="N", help="force annealing at specified epoch")
        group.add_argument("--warmup-updates", default=0, type=int, metavar="N",
                           help="warmup the learning rate linearly for the first N updates")
        group.add_argument("--end-learning-rate", default=0.0, type=float)
        group.add_argument("--power", default=1.0, type=float)
        group.add_argument("--total-num-update", default=1000000, type=int)
    else:
        raise ValueError("unsupported lr_scheduler: {}".format(lr_scheduler))
    return group


def add_checkpoint_args(parser):
    group = parser.add_argument_group("Checkpointing")
    group.add_argument("--save-dir", metavar="DIR", default="checkpoints", help="path to save checkpoints")
    group.add_argument("--restore-file", default="checkpoint_last.pt",
                       help="filename from which to load checkpoint (default: <save-dir>/checkpoint_last.pt")
    group.add_argument("--reset-dataloader", action="store_true",
                       help="if set, does not reload dataloader state from the checkpoint")
    group.add_argument("--reset-lr-scheduler", action="store_true",
                       help="if set, does not load lr scheduler state from the checkpoint")
    group.add_argument("--reset-meters", action="store_true", help="if set, does not load meters from the checkpoint")
    group.add_argument("--reset-optimizer", action="store_true",
                       help="if set, does not load optimizer state from the checkpoint")
    group.add_argument("--optimizer-overrides", default="{}", type=str, metavar="DICT",
                       help="a dictionary used to override optimizer args when loading a checkpoint")
    group.add_argument("--save-interval", type=int, default=1, metavar="N", help="save a checkpoint every N epochs")
    group.add_argument("--save-interval-updates", type=int, default=0, metavar="N",
                       help="save a checkpoint every N updates")
    group.add_argument("--keep-interval-updates", type=int, default=-1, metavar="N",
                       help="keep the last N checkpoints saved with --save-interval-updates")
    group.add_argument("--keep-last-epochs", type=int, default=-1, metavar="N", help="keep last N epoch checkpoints")
    group.add_argument("--no-save", action="store_true", help="don't save models or checkpoints")
    group.add_argument("--no-epoch-checkpoints", action="store_true", help="only store last and best checkpoints")
    group.add_argument("--no-last-checkpoints", action="store_true", help="don't store last checkpoints")
    group.add_argument("--no-save-optimizer-state", action="store_true",
                       help="don't save optimizer-state as part of checkpoint")
    group.add_argument("--best-checkpoint-metric", type=str, default="loss",
                       help='metric to use for saving "best" checkpoints')
    group.add_argument("--maximize-best-checkpoint-metric", action="store_true",
                       help='select the largest metric value for saving "best" checkpoints')
    return group


def add_mi355x_args(parser):
    group = parser.add_argument_group("MI355X runtime (extensions)")
    group.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                       help="compute dtype: fp32 (reference parity) or bf16 MFMA with fp32 master weights")
    group.add_argument("--fp32-gemm", default=None, choices=["h3p", "h3", "x6", "native"],
                       help="fp32 GEMM engine (default h3p; HETSEQ_FP32_GEMM): h3p = the encoder and head on "
                            "pre-split fp16 planes with a power-of-two exponent per 32 x 32 block, h3 elsewhere; "
                            "h3 = three split-fp16 products with per-tensor power-of-two scales; x6 = six "
                            "split-bf16 products, no scale (fp32-level error at any range); native = exact-fp32 "
                            "MFMA")
    group.add_argument("--fused", dest="fused", action="store_true", default=True,
                       help="use the gfx950 HIP kernel path on GPU (default)")
    group.add_argument("--no-fused", dest="fused", action="store_false", help="use the torch-op reference path")
    group.add_argument("--device-id-offset", type=int, default=0,
                       help="local process i uses device i+offset (heterogeneous launches sharing one node)")
    group.add_argument("--per-rank-seed", action="store_true",
                       help="seed dropout with seed+num_updates+rank (reference uses the same seed on all ranks)")
    group.add_argument("--check-consistency", type=int, default=0, metavar="N",
                       help="every N updates all-reduce a parameter checksum and fail on divergence")
    group.add_argument("--comm-channels", type=int, default=None, metavar="N",
                       help="cap RCCL's channels (NCCL_MAX_NCHANNELS) for the gradient collectives: each channel "
                            "holds a workgroup slot beside the backward's GEMMs (profiles/r4_dp_emulation.md)")
    group.add_argument("--emulate-world", type=int, default=None, metavar="W", help=argparse.SUPPRESS)
    group.add_argument("--collective-timeout", type=float, default=1800.0, metavar="SEC",
                       help="timeout for process-group collectives; the native engine's watchdog aborts the "
                            "communicator when a collective outlives it")
    group.add_argument("--comm-engine", default="auto", choices=["auto", "native", "c10d"],
                       help="gradient / stats collectives: the native RCCL engine (greatest-priority comm "
                            "stream, event-gated buckets, watchdog; auto = on GPUs with the nccl backend) or "
                            "torch.distributed (c10d)")
    group.add_argument("--shard-optimizer", default="auto", choices=["auto", "on", "off"],
                       help="data-parallel Adam: reduce-scatter the gradient buckets, update 1/W of the parameters "
                            "per rank and all-gather them layer by layer beside the next forward "
                            "(parallel/zero.py; auto = on for data-parallel Adam runs without BMUF / HIP graphs on "
                            "the native RCCL engine, after its in-place collectives pass a self-test on the job's "
                            "ranks; on = also with c10d)")
    group.add_argument("--no-sparse-embedding-exchange", dest="sparse_embedding_exchange", action="store_false",
                       help="all-reduce the embedding tables densely in the last bucket instead of the early "
                            "dense bucket (tied decoder part) + all-gather of the per-token rows")
    group.add_argument("--checkpoint-activations", action="store_true",
                       help="recompute encoder layers during backward to save activation memory")
    group.add_argument("--json-log", type=str, default=None, metavar="PATH",
                       help="append one JSON object per logged update")
    group.add_argument("--profile", action="store_true", help="roctx ranges and per-phase hipEvent timing")
    group.add_argument("--hip-graph", action="store_true",
                       help="capture the whole update (forward, backward, clip, Adam) in a HIP graph after a few "
                            "eager warm-up updates and replay it (single process, --fast-stat-sync, update-freq 1)")
    group.add_argument("--deterministic", action="store_true",
                       help="bitwise-reproducible mode: deterministic torch algorithms, fixed RCCL ring/simple "
                            "protocol, no tuned GEMM table (library split-K solutions may use atomics)")
    group.add_argument("--no-gemm-tuning", dest="gemm_tuning", action="store_false",
                       help="do not load the measured hipBLASLt/rocBLAS GEMM table (configs/tunableop)")
    group.add_argument("--gemm-tune-missing", action="store_true",
                       help="let TunableOp time library GEMM shapes missing from the table on first use "
                            "(off by default: live tuning runs untested candidate solutions mid-training)")
    group.add_argument("--bmuf-block-momentum", type=float, default=0.875,
                       help="block momentum for --use-bmuf")
    group.add_argument("--bmuf-sync-interval", type=int, default=1,
                       help="updates between BMUF model synchronisations")
    return group


def eval_str_list(x, type=float):
    if x is None:
        return None
    if isinstance(x, str):
        x = ast.literal_eval(x)
    try:
        return list(map(type, x))
    except TypeError:
        return [type(x)]


def eval_bool(x, default=False):
    if x is None:
        return default
    try:
        return bool(ast.literal_eval(x))
    except (TypeError, ValueError):
        return default


def parse_args_and_arch(parser, s=None):
    args = parser.parse_args(s)
    if hasattr(args, "max_sentences_valid") and args.max_sentences_valid is None:
        args.max_sentences_valid = args.max_sentences
    if hasattr(args, "max_tokens_valid") and args.max_tokens_valid is None:
        args.max_tokens_valid = args.max_tokens
    return args


def get_pre_parser():
    p = argparse.ArgumentParser(allow_abbrev=False, add_help=False)
    p.add_argument("--task", type=str, default="bert", choices=["bert", "mnist"])
    p.add_argument("--optimizer", type=str, default="adam", choices=["adam", "adadelta", "lamb"])
    p.add_argument("--lr-scheduler", type=str, default="PolynomialDecayScheduler",
                   choices=["PolynomialDecayScheduler"])
    return p


def parse_cli(argv=None):
    """Two-stage parse (reference: train.py:197-211)."""
    pre, rest = get_pre_parser().parse_known_args(argv)
    parser = get_training_parser(task=pre.task, optimizer=pre.optimizer, lr_scheduler=pre.lr_scheduler)
    # the full parser re-declares --task/--optimizer; feed them back in
    rest = list(rest) + ["--task", pre.task, "--optimizer", pre.optimizer]
    return parse_args_and_arch(parser, rest)
