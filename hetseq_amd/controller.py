"""Controller: the synchronous data-parallel training engine.

API parity with the reference ``Controller`` (reference: controller.py:21-438):
``model``/``optimizer``/``lr_scheduler`` properties, ``train_step(samples)``,
``get_train_iterator``, ``save_checkpoint``/``load_checkpoint``,
``lr_step``/``lr_step_update``/``get_lr``, meters, ``get/set_num_updates``.
Reference semantics kept on purpose: per-update reseeding
with ``seed + num_updates`` (Q14), ``sample_size = len(sample[0][0])`` grad
normalisation (Q03), fast-stat loss units ``sum loss / (sum sample_size *
ln 2)`` (Q02), dummy batch with ``loss * 0`` for padded shards (C26), grad
clipping at ``--clip-norm``.

MI355X-first engine underneath:
* parameters/gradients live in a flat store; DP uses ``FlatDDP`` (in-place
  bucketed all-reduce on RCCL, overlapped with backward) instead of DDP;
* the whole update (grad scale, clip, Adam) is one reduction + one fused
  kernel reading the scale from device memory -- the stats all-reduce
  result never round-trips to the host inside ``train_step``;
* meters take device tensors lazily, so with logging off a training step
  issues no host synchronisation at all (the reference syncs 3-4 times per
  update);
* ``--dtype bf16`` keeps fp32 master weights and a bf16 shadow copy.
"""
from __future__ import annotations

import contextlib
import math
import os
from collections import OrderedDict
from itertools import chain

import torch
import torch.distributed as dist

from hetseq_amd import checkpoint_utils, utils
from hetseq_amd.meters import AverageMeter, StopwatchMeter, TimeMeter
from hetseq_amd.ops._C import hip, stream_handle
from hetseq_amd.optim import build_lr_scheduler, build_optimizer
from hetseq_amd.parallel import distributed_utils
from hetseq_amd.parallel.ddp import BMUF, FlatDDP
from hetseq_amd.runtime import faults, profiling, rng, streams
from hetseq_amd.runtime.flat import FlatParamStore

# zero_grad clears only the gradient regions the next backward does not overwrite (HETSEQ_LAZY_ZERO=0: all)
_LAZY_ZERO = os.environ.get("HETSEQ_LAZY_ZERO", "1") == "1"
# staged update: the optimizer step runs chunk by chunk on its own stream, overlapped with the next
# forward (optim/optimizers.py; one GPU, eager steps, models that declare update chunks).
# HETSEQ_STAGED_UPDATE=0: the whole update before the next step.
STAGED_UPDATE = os.environ.get("HETSEQ_STAGED_UPDATE", "1") == "1"

LN2 = math.log(2)


class Controller(object):
    def __init__(self, args, task, model, criterion=None, dummy_batch=None, oom_batch=None):
        self.args = args
        self.task = task
        self.cuda = torch.cuda.is_available() and not args.cpu
        self.device = torch.device("cuda", torch.cuda.current_device()) if self.cuda else torch.device("cpu")
        self._model = model.to(self.device)
        if not getattr(args, "fused", True):
            os.environ["HETSEQ_DISABLE_FUSED"] = "1"
        self.compute_dtype = torch.bfloat16 if getattr(args, "dtype", "fp32") == "bf16" else torch.float32
        # weight-gradient side stream (runtime/streams.py): on for the GEMM-bound fp32 step
        # (BERT-base 18.4 -> 16.6 ms); off for bf16, whose eager step is host-bound (the stream
        # switches cost ~1 ms of host time per step there) and under --hip-graph (HIP graph
        # replay does not run the two branches concurrently).  HETSEQ_WGRAD_STREAM overrides.
        if getattr(args, "fp32_gemm", None):
            from hetseq_amd.ops import gemm as G

            G.set_fp32_mode(args.fp32_gemm)
        if "HETSEQ_WGRAD_STREAM" not in os.environ:
            streams.set_enabled(self.compute_dtype == torch.float32 and not getattr(args, "hip_graph", False))
        # library-GEMM tables (TunableOp) are process-global: loaded by the entry points
        # (train.py / bench.py -> runtime.gemm_tuning.configure), never here
        shadow = torch.bfloat16 if self.compute_dtype == torch.bfloat16 else None
        self.store = FlatParamStore(self._model, device=self.device, shadow_dtype=shadow)
        if hasattr(self._model, "attach_store"):
            self._model.attach_store(self.store, self.compute_dtype)
        elif self.compute_dtype != torch.float32:
            raise ValueError("--dtype bf16 is only implemented for the BERT models")
        self._dummy_batch = dummy_batch
        self._oom_batch = oom_batch or dummy_batch
        self._lr_scheduler = None
        self._num_updates = 0
        self._optim_history = None
        self._optimizer = None
        self._prev_grad_norm = None
        self._wrapped_model = None
        self._bmuf = None
        self._all_reduce_list = [0.0] * 6
        self.fast_stat_sync = args.fast_stat_sync
        self.phase_timer = profiling.PhaseTimer()
        self._graph = None  # runtime.graphs.GraphedStep once --hip-graph captured the update
        self._scale_buf = None  # fp32 device scalar: the gradient scale of the fast-stat path
        self._graph_warmup = 3  # eager updates first: GEMM autotuning, TunableOp, allocator warm-up
        self.init_meters(args)

    def init_meters(self, args):
        self.meters = OrderedDict()
        self.meters["train_loss"] = AverageMeter()
        self.meters["train_nll_loss"] = AverageMeter()
        self.meters["valid_loss"] = AverageMeter()
        self.meters["valid_nll_loss"] = AverageMeter()
        self.meters["wps"] = TimeMeter()
        self.meters["ups"] = TimeMeter()
        self.meters["wpb"] = AverageMeter()
        self.meters["bsz"] = AverageMeter()
        self.meters["gnorm"] = AverageMeter()
        self.meters["clip"] = AverageMeter()
        self.meters["wall"] = TimeMeter()
        self.meters["train_wall"] = StopwatchMeter()

    # ------------------------------------------------------------------ properties
    @property
    def model(self):
        if self._wrapped_model is None:
            multi = self.args.distributed_world_size > 1 or getattr(self.args, "force_ddp", False)
            if multi and dist.is_initialized() and not self.args.use_bmuf:
                sparse, cap = self._sparse_embedding()
                self._wrapped_model = FlatDDP(self._model, self.store, bucket_cap_mb=self.args.bucket_cap_mb,
                                              find_unused_parameters=self.args.find_unused_parameters,
                                              comm_engine=getattr(self.args, "comm_engine", "auto"),
                                              timeout_s=getattr(self.args, "collective_timeout", 1800.0),
                                              sparse_embedding=sparse, sparse_capacity=cap,
                                              plan_world=getattr(self.args, "emulate_world", None),
                                              shard_optimizer=self._shard_ok())
            else:
                self._wrapped_model = self._model
                if self.args.distributed_world_size > 1 and dist.is_initialized() and self.args.use_bmuf:
                    self._bmuf = BMUF(self.store, block_momentum=self.args.bmuf_block_momentum,
                                      sync_interval=self.args.bmuf_sync_interval)
        return self._wrapped_model

    def _sparse_embedding(self):
        """Embedding tables the data-parallel engine exchanges sparsely (parallel/tied.py), when the
        model declares them and the fused BERT path (the only one handing rows over) is on, and the
        row capacity per micro-batch: the configured bound (``--max-sentences`` x the training data's
        sequence length, or ``--max-tokens``), identical on every rank by construction, so no batch
        can overflow it on one rank only.  (None, None) when no bound is known: dense tables."""
        fn = getattr(self._model, "sparse_embedding", None)
        if fn is None or getattr(self.args, "sparse_embedding_exchange", True) is False:
            return None, None
        ds = getattr(self.task, "datasets", {}).get(getattr(self.args, "train_subset", "train"))
        S = getattr(ds, "seq_len", None)
        cap = None
        if getattr(self.args, "max_sentences", None) and S:
            cap = int(self.args.max_sentences) * int(S)
        elif getattr(self.args, "max_tokens", None):
            cap = int(self.args.max_tokens)
        if cap is None:
            return None, None
        return fn(), cap

    @property
    def optimizer(self):
        if self._optimizer is None:
            self._build_optimizer()
        return self._optimizer

    @property
    def lr_scheduler(self):
        if self._lr_scheduler is None:
            self._build_optimizer()
        return self._lr_scheduler

    def _build_optimizer(self):
        params = list(filter(lambda p: p.requires_grad, chain(self.model.parameters())))
        self._optimizer = build_optimizer(self.args, params, self.store)
        self._optimizer.staged = self._staged_ok()
        self._lr_scheduler = build_lr_scheduler(self.args, self._optimizer)
        self._lr_scheduler.step_update(0)

    def _shard_ok(self):
        """Sharded optimizer (parallel/zero.py): data-parallel Adam runs (the flat-store update with a
        range form), eager steps, no BMUF.  "auto" (default): the data-parallel engine shards on the
        native RCCL engine once its self-test passed (parallel/comm.py shard_self_test); "on" shards on
        any engine; "off" never."""
        mode = getattr(self.args, "shard_optimizer", "auto")
        ok = (mode != "off" and getattr(self.args, "optimizer", "adam") == "adam"
              and not getattr(self.args, "hip_graph", False) and not self.args.use_bmuf)
        return ("auto" if mode == "auto" else True) if ok else False

    def _staged_ok(self):
        """Staged (overlapped) update: eager steps (a HIP graph replays the whole update) of a model
        whose forward waits per chunk (runtime/flat.py set_chunks), on one GPU (its own update stream)
        or with the sharded data-parallel update on the native engine (the update and the chunks'
        all-gathers on the comm stream); a data-parallel step's collectives and a fifth stream would
        share hardware queues."""
        if not (STAGED_UPDATE and self.cuda and self.store.chunks is not None and not getattr(self.args, "hip_graph", False)):
            return False
        if not (self.args.distributed_world_size > 1 or getattr(self.args, "force_ddp", False)):
            return True
        m = self.model
        return getattr(m, "shard", None) is not None and getattr(m, "comm", None) is not None

    # ------------------------------------------------------------------ checkpoints
    def consolidate_optimizer(self):
        """Every rank, before the master's save: the sharded optimizer's state gathered whole."""
        if self._optimizer is not None:
            self._optimizer.consolidate()

    def save_checkpoint(self, filename, extra_state):
        self.store.params_ready()
        if distributed_utils.is_master(self.args):
            extra_state["train_meters"] = self.meters
            checkpoint_utils.save_state(filename, self.args, self.get_model().state_dict(), None, self.optimizer,
                                        self.lr_scheduler, self.get_num_updates(), self._optim_history, extra_state)

    def load_checkpoint(self, filename, reset_optimizer=False, reset_lr_scheduler=False, optimizer_overrides=None,
                        reset_meters=False):
        extra_state, self._optim_history, last_optim_state = None, [], None
        if os.path.exists(filename):
            state = checkpoint_utils.load_checkpoint_to_cpu(filename)
            try:
                self.get_model().load_state_dict(state["model"], strict=True)
            except Exception:
                raise Exception("Cannot load model parameters from checkpoint {}; please ensure that the "
                                "architectures match.".format(filename))
            self.store.sync_shadow()
            extra_state = state["extra_state"]
            self._optim_history = state["optimizer_history"]
            last_optim_state = state.get("last_optimizer_state", None)
        if last_optim_state is not None and not reset_optimizer:
            self._build_optimizer()
            last_optim = self._optim_history[-1]
            assert last_optim["optimizer_name"] == self.optimizer.__class__.__name__, \
                "Optimizer does not match; please reset the optimizer (--reset-optimizer)."
            if not reset_lr_scheduler:
                self.lr_scheduler.load_state_dict(last_optim["lr_scheduler_state"])
            self.optimizer.load_state_dict(last_optim_state, optimizer_overrides)
            self.set_num_updates(last_optim["num_updates"])
        if extra_state is not None:
            itr = extra_state.get("train_iterator", {"epoch": 0})
            epoch = itr["epoch"]
            print("| loaded checkpoint {} (epoch {} @ {} updates)".format(filename, epoch, self.get_num_updates()))
            self.lr_step(epoch)
            if "train_meters" in extra_state and not reset_meters:
                checkpoint_utils.restore_meters(self.meters, extra_state["train_meters"])
                del extra_state["train_meters"]
                for meter in self.meters.values():
                    if isinstance(meter, TimeMeter):
                        meter.reset()
        else:
            print("| no existing checkpoint found {}".format(filename))
        return extra_state

    def checkpoint_num_updates(self):
        """Update count recorded in the loaded checkpoint's optimizer history (0 if none) -- also
        under --reset-optimizer, where the controller's own count restarts at 0."""
        return int(self._optim_history[-1].get("num_updates", 0)) if self._optim_history else 0

    def get_train_iterator(self, epoch, combine=True, load_dataset=True):
        if load_dataset:
            print("| loading train data for epoch {}".format(epoch))
            self.task.load_dataset(self.args.train_subset)
        return self.task.get_batch_iterator(
            dataset=self.task.dataset(self.args.train_subset), max_tokens=self.args.max_tokens,
            max_sentences=self.args.max_sentences, max_positions=None, ignore_invalid_inputs=True,
            required_batch_size_multiple=self.args.required_batch_size_multiple, seed=self.args.seed,
            num_shards=self.args.distributed_world_size, shard_id=self.args.distributed_rank,
            num_workers=self.args.num_workers, epoch=epoch, device=self.device if self.cuda else None)

    # ------------------------------------------------------------------ training
    def train_step(self, samples, dummy_batch=False, raise_oom=False):
        """Forward, backward and parameter update for one group of micro-batches."""
        if self._graph_eligible(samples, dummy_batch):
            out = self._train_step_graphed(samples[0])
            if out is not None:
                return out
        if self._dummy_batch is None:
            self._dummy_batch = next((s for s in samples if s is not None and len(s) > 0), None)
        faults.maybe_inject(getattr(self.args, "distributed_rank", 0) or 0, self._num_updates)
        self._set_seed()
        if not self._model.training:
            self.model.train()  # (a recursive walk over every module: only when the mode changes)
        self.zero_grad()
        if not dummy_batch:
            self.meters["train_wall"].start()
        logging_outputs, sample_sizes, ooms = [], [], 0
        stats = torch.zeros(6, dtype=torch.float64, device=self.device) if self.fast_stat_sync else None
        sample_size = 0
        logging_output = {}
        for i, sample in enumerate(samples):
            sample = self._prepare_sample(sample)
            if sample is None:
                sample = self._prepare_sample(self._dummy_batch)
                ignore_grad = True
            else:
                ignore_grad = False

            def maybe_no_sync():
                if self.args.distributed_world_size > 1 and hasattr(self.model, "no_sync") and i < len(samples) - 1:
                    return self.model.no_sync()
                return contextlib.ExitStack()

            try:
                with maybe_no_sync():
                    tok = self.phase_timer.start("fwd_bwd")
                    loss, sample_size, logging_output = self.task.train_step(sample, self.model, self.optimizer,
                                                                             ignore_grad)
                    self.phase_timer.stop(tok)
                if not ignore_grad:
                    logging_outputs.append(logging_output)
                    sample_sizes.append(sample_size)
                    if self.fast_stat_sync and not _stats_accum_fused(stats, sample_size, logging_output):
                        stats[0] += sample_size
                        stats[1] += logging_output.get("nsentences", 0.0)
                        stats[2] += _as_f64(logging_output.get("loss", 0.0), self.device)
                        stats[3] += _as_f64(logging_output.get("nll_loss", 0.0), self.device)
                        stats[4] += logging_output.get("ntokens", 0.0)
            except RuntimeError as e:
                if "out of memory" in str(e):
                    raise RuntimeError("ran out of memory with exception") from e
                raise e
        if dummy_batch:
            return None

        scale = None  # grad multiplier: W/sample_size of the reference, divided by W (we sum, not average)
        if self.fast_stat_sync:
            if self._sync_stats():
                if isinstance(self.model, FlatDDP):
                    self.model.all_reduce_(stats)  # native engine: in-stream RCCL, no c10d bookkeeping
                else:
                    dist.all_reduce(stats)
            w = 1.0 if isinstance(self.model, FlatDDP) else float(self.args.distributed_world_size)
            if stats.is_cuda:  # one launch: division + gradient scale (the step's tail is host-bound)
                if self._scale_buf is None:
                    self._scale_buf = torch.empty(1, dtype=torch.float32, device=stats.device)
                hip().stats_finalize(stats.data_ptr(), LN2, w, self._scale_buf.data_ptr(), stream_handle())
                scale = self._scale_buf[0]
            else:
                stats[2:4].div_(stats[0:1] * LN2)
                scale = torch.where(stats[0] > 0, w / stats[0].clamp(min=1e-30), torch.ones_like(stats[0])).float()
            sample_size_t = stats[0]
            logging_output = {"nsentences": stats[1], "loss": stats[2], "nll_loss": stats[3], "ntokens": stats[4]}
            ooms = stats[5]
            sample_size_for_meter = sample_size_t
        else:
            if self._sync_stats():
                gathered = distributed_utils.all_gather_list(
                    [_to_host(logging_outputs), sample_sizes, ooms, _host(self._prev_grad_norm)])
                logging_outputs_all, sample_sizes_all, ooms_all, prev_norms = zip(*gathered)
                ooms = sum(ooms_all)
                if not self.args.use_bmuf:
                    assert (all(n == prev_norms[0] for n in prev_norms)
                            or all(n is None or math.isnan(n) or math.isinf(n) for n in prev_norms)), \
                        "Fatal error: gradients are inconsistent between workers"
            if sample_size > 0:
                # reference: W/sample_size applied to DDP-averaged grads == 1/sample_size on summed grads
                scale = 1.0 / float(sample_size)
                if not (self.args.distributed_world_size > 1 and dist.is_initialized() and not self.args.use_bmuf):
                    scale = float(self.args.distributed_world_size) / float(sample_size)
            sample_size_for_meter = sample_size
        if not all(k in logging_output for k in ["ntokens", "nsentences"]):
            raise Exception("Please update the {}.aggregate_logging_outputs() method to return ntokens and "
                            "nsentences".format(self.task.__class__.__name__))
        try:
            tok = self.phase_timer.start("optimizer")
            profiling.range_push("optimizer")
            if scale is not None:
                self.optimizer.multiply_grads(scale)
            grad_norm = self.optimizer.clip_grad_norm(self.args.clip_norm)
            self._prev_grad_norm = grad_norm
            self.optimizer.step()
            if self._bmuf is not None:
                self._bmuf.after_step()
            profiling.range_pop()
            self.phase_timer.stop(tok)
            self.set_num_updates(self.get_num_updates() + 1)
            self.task.update_step(self._num_updates)
            ntokens = logging_output.get("ntokens", 0)
            nsentences = logging_output.get("nsentences", 0)
            self.meters["wps"].update(ntokens)
            self.meters["ups"].update(1.0)
            self.meters["wpb"].update(ntokens)
            self.meters["bsz"].update(nsentences)
            self.meters["gnorm"].update(grad_norm)
            if self.args.clip_norm > 0:
                self.meters["clip"].update((grad_norm > self.args.clip_norm).float() if torch.is_tensor(grad_norm)
                                           else float(grad_norm > self.args.clip_norm))
            else:
                self.meters["clip"].update(0.0)
            self.meters["train_loss"].update(logging_output.get("loss", 0), sample_size_for_meter)
            if self.args.check_consistency and self._num_updates % self.args.check_consistency == 0:
                self.check_consistency()
        except OverflowError as e:
            print("| WARNING: overflow detected, " + str(e))
            self.zero_grad()
            logging_output = None
        self.clear_buffered_stats()
        self.meters["train_wall"].stop()
        return logging_output

    # ------------------------------------------------------------------ HIP graph path
    def _graph_eligible(self, samples, dummy_batch):
        a = self.args
        # data-parallel runs capture too when the gradients go through the native RCCL engine: its
        # collectives are enqueued on streams (captured into the graph, replayed in the same order
        # on every rank); c10d / gloo and BMUF stay eager
        # (c10d / gloo: the collectives cannot be captured, so forward+backward and the update are
        # two graphs with the gradient exchange between them -- _graph_split)
        dp = self._sync_stats() or isinstance(self.model, FlatDDP)
        dp_ok = not dp or (isinstance(self.model, FlatDDP) and not a.use_bmuf)
        return (getattr(a, "hip_graph", False) and self.cuda and self.fast_stat_sync and not dummy_batch
                and len(samples) == 1 and samples[0] is not None and len(samples[0]) > 0 and dp_ok
                and getattr(self.optimizer, "supports_device_hyper", False)
                and self._num_updates >= self._graph_warmup)

    def _graph_body(self, sample):
        """The captured update (fast-stat path of train_step; data-parallel: the bucket, table and
        statistics collectives of the native engine are captured with it)."""
        self.zero_grad()
        stats = torch.zeros(6, dtype=torch.float64, device=self.device)
        _, sample_size, lo = self.task.train_step(sample, self.model, self.optimizer, False)
        stats[0] += sample_size
        stats[1] += lo.get("nsentences", 0.0)
        stats[2] += _as_f64(lo.get("loss", 0.0), self.device)
        stats[3] += _as_f64(lo.get("nll_loss", 0.0), self.device)
        stats[4] += lo.get("ntokens", 0.0)
        if self._sync_stats():
            self.model.all_reduce_(stats)  # in-stream RCCL (captured)
        stats[2:4].div_(stats[0:1] * LN2)
        scale = torch.where(stats[0] > 0, 1.0 / stats[0].clamp(min=1e-30), torch.ones_like(stats[0])).float()
        self.optimizer.multiply_grads(scale)
        grad_norm = self.optimizer.clip_grad_norm(self.args.clip_norm)
        self.optimizer.step(launch_only=True)
        return stats, grad_norm.reshape(1)

    def _graph_split(self):
        """Data-parallel through torch.distributed (c10d / gloo): collectives cannot be captured."""
        return isinstance(self.model, FlatDDP) and self.model.comm is None

    def _graph_fwd_bwd(self, sample):
        """Split graph 1: forward + backward with no collective (gradients stay local)."""
        self.zero_grad()
        stats = torch.zeros(6, dtype=torch.float64, device=self.device)
        with self.model.no_sync():
            _, sample_size, lo = self.task.train_step(sample, self.model, self.optimizer, False)
        stats[0] += sample_size
        stats[1] += lo.get("nsentences", 0.0)
        stats[2] += _as_f64(lo.get("loss", 0.0), self.device)
        stats[3] += _as_f64(lo.get("nll_loss", 0.0), self.device)
        stats[4] += lo.get("ntokens", 0.0)
        return (stats,)

    def _graph_update(self, inputs):
        """Split graph 2: the update from the exchanged gradients and statistics."""
        stats = inputs[0]
        stats[2:4].div_(stats[0:1] * LN2)
        scale = torch.where(stats[0] > 0, 1.0 / stats[0].clamp(min=1e-30), torch.ones_like(stats[0])).float()
        self.optimizer.multiply_grads(scale)
        grad_norm = self.optimizer.clip_grad_norm(self.args.clip_norm)
        self.optimizer.step(launch_only=True)
        return stats, grad_norm.reshape(1)

    def _run_split_graphs(self, sample):
        g1, g2 = self._graph
        (stats,) = g1.run(list(sample))
        self.model.all_reduce_grads()  # eager c10d exchange of the flat gradient buffer
        self.model.all_reduce_(stats)
        return g2.run([stats])

    def _end_failed_capture(self):
        """A failed capture can leave streams that joined it (the side stream, through an event wait)
        still capturing, and an error pending that the next launch reports: end those captures so
        the eager fallback runs."""
        handles = set(streams.engine_streams(self.device).values())
        handles.add(torch.cuda.current_stream(self.device).cuda_stream)
        for h in handles:
            was, err = hip().end_capture(h)
            if was or err:
                print("| ended the failed capture of stream {:#x} (pending HIP error {})".format(h, err), flush=True)
        torch.cuda.synchronize(self.device)

    def _train_step_graphed(self, sample):
        from hetseq_amd.runtime.graphs import GraphedStep

        sample = self._prepare_sample(sample)
        if self._graph is False:
            return None  # capture failed once: stay eager
        split = self._graph_split()
        if self._graph is None:
            rng.enable_device_seed(self.device)
            self.optimizer.enable_device_hyper(self.device)
            comm = getattr(self.model, "comm", None)
            if split:
                self._graph = (GraphedStep(self._graph_fwd_bwd), GraphedStep(self._graph_update))
            else:
                # with a communicator the watchdog thread queries events during capture: errors of
                # other threads must not invalidate it (thread-local capture mode)
                self._graph = GraphedStep(self._graph_body, capture_error_mode="thread_local" if comm else "global")
        elif not (self._graph[0] if split else self._graph).matches(sample):
            return None  # e.g. a short last batch: run it eagerly
        faults.maybe_inject(getattr(self.args, "distributed_rank", 0) or 0, self._num_updates)
        self._set_seed()
        self.optimizer.graph_prepare()
        self.meters["train_wall"].start()
        try:
            stats, grad_norm = self._run_split_graphs(sample) if split else self._graph.run(list(sample))
        except RuntimeError as e:
            first = self._graph[0] if split else self._graph
            if first.graph is not None and first.static_out is not None:
                raise  # a replay failure (or a failure after the first graph ran) is a real error
            # capture failed (nothing ran): undo the host half of the update and fall back to eager
            print("| WARNING: HIP graph capture failed ({}); continuing eagerly".format(str(e).splitlines()[0]),
                  flush=True)
            if os.environ.get("HETSEQ_CAPTURE_DEBUG") == "1":
                import traceback

                traceback.print_exc()
            self._end_failed_capture()
            self.optimizer.step_count -= 1
            self._graph = False
            return None
        comm = getattr(self.model, "comm", None)
        if comm is not None:
            comm.watch()  # the replayed collectives under the watchdog
            comm.check()
        grad_norm = grad_norm[0]
        self.set_num_updates(self.get_num_updates() + 1)
        self.task.update_step(self._num_updates)
        logging_output = {"nsentences": stats[1], "loss": stats[2], "nll_loss": stats[3], "ntokens": stats[4]}
        self._prev_grad_norm = grad_norm
        self.meters["wps"].update(stats[4])
        self.meters["ups"].update(1.0)
        self.meters["wpb"].update(stats[4])
        self.meters["bsz"].update(stats[1])
        self.meters["gnorm"].update(grad_norm)
        self.meters["clip"].update((grad_norm > self.args.clip_norm).float() if self.args.clip_norm > 0 else 0.0)
        self.meters["train_loss"].update(stats[2], stats[0])
        if self.args.check_consistency and self._num_updates % self.args.check_consistency == 0:
            self.check_consistency()
        self.meters["train_wall"].stop()
        return logging_output

    def check_consistency(self):
        """All-reduce the parameter checksum and fail if ranks diverged."""
        if not (dist.is_initialized() and self.args.distributed_world_size > 1) or self.args.use_bmuf:
            return
        cs = self.store.checksum().reshape(1)
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        if float(hi - lo) > 1e-6 * max(1.0, abs(float(cs))):
            raise RuntimeError("parameter checksum diverged across ranks: min {} max {}".format(float(lo), float(hi)))

    def zero_grad(self):
        # lazy: the fused backward overwrites most of the gradient buffer (runtime/flat.py cover())
        self.optimizer.zero_grad(lazy=_LAZY_ZERO and self.cuda)

    def clear_buffered_stats(self):
        self._all_reduce_list = [0.0] * 6

    def lr_step(self, epoch, val_loss=None):
        self.lr_scheduler.step(epoch, val_loss)
        return self.lr_step_update()

    def lr_step_update(self):
        return self.lr_scheduler.step_update(self.get_num_updates())

    def get_lr(self):
        return self.optimizer.get_lr()

    def get_model(self):
        return self._model

    def get_meter(self, name):
        return self.meters.get(name)

    def get_num_updates(self):
        return self._num_updates

    def set_num_updates(self, num_updates):
        self._num_updates = num_updates
        self.lr_step_update()

    def _prepare_sample(self, sample):
        if sample is None or len(sample) == 0:
            return None
        if self.cuda:
            sample = utils.move_to_cuda(sample, self.device)
        return sample

    def _set_seed(self):
        seed = self.args.seed + self.get_num_updates()
        if getattr(self.args, "per_rank_seed", False):
            seed += 1000003 * int(self.args.distributed_rank or 0)
        torch.manual_seed(seed)
        if self.cuda:
            torch.cuda.manual_seed(seed)
        rng.set_seed(seed)

    def _sync_stats(self):
        return self.args.distributed_world_size > 1 and dist.is_initialized()


def _stats_accum_fused(stats, sample_size, lo):
    """stats[0..4] += this micro-batch's (sample_size, nsentences, loss, nll_loss, ntokens) in one HIP
    launch when the losses are fp32 device scalars and the counts host numbers; False otherwise."""
    if stats is None or not stats.is_cuda:
        return False
    vals = [lo.get("nsentences", 0.0), lo.get("ntokens", 0.0), sample_size]
    losses = [lo.get("loss", 0.0), lo.get("nll_loss", 0.0)]
    if any(torch.is_tensor(v) for v in vals):
        return False
    for t in losses:
        if not (torch.is_tensor(t) and t.is_cuda and t.dtype == torch.float32 and t.numel() == 1
                and t.is_contiguous() and t.device == stats.device):
            return False
    hip().stats_accum(stats.data_ptr(), losses[0].data_ptr(), losses[1].data_ptr(), float(sample_size),
                      float(vals[0]), float(vals[1]), stream_handle())
    return True


def _as_f64(v, device):
    if torch.is_tensor(v):
        return v.detach().to(device=device, dtype=torch.float64)
    return float(v)


def _host(v):
    if torch.is_tensor(v):
        return float(v.item())
    return v


def _to_host(logging_outputs):
    return [{k: _host(v) for k, v in lo.items()} for lo in logging_outputs]
