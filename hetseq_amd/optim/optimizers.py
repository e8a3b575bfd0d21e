"""Optimizers over the flat parameter store.

API parity with the reference wrappers (reference: optim.py:6-131):
``_Optimizer`` with ``get_lr/set_lr``, ``state_dict/load_state_dict`` (with
``optimizer_overrides``), ``backward``, ``multiply_grads``,
``clip_grad_norm`` and ``step``/``zero_grad``; ``_Adam`` (fairseq AdamW
semantics, Q16/Q20) and ``_Adadelta``; plus ``_Lamb`` (extension).  Class
names are kept so checkpoints record the same ``optimizer_name``.

Execution model (MI355X-first):
  multiply_grads(c)  -> records c (host float or 0-d device tensor); grads untouched
  clip_grad_norm(m)  -> one reduction kernel over the flat grad buffer; the total
                        norm of c*g and the combined multiplier c*clip stay on
                        device (returned norm is a 0-d device tensor)
  step()             -> ONE fused kernel: reads g*multiplier, updates p/m/v (and
                        the bf16 shadow copy) in place
No host synchronisation happens anywhere in the update.  On CPU the same
math runs as a handful of vectorised torch ops over the flat buffers.

``state_dict`` is the ``torch.optim`` layout (``state[i] = {step, exp_avg,
exp_avg_sq}``, ``param_groups`` with lr/betas/eps/weight_decay/amsgrad) with
parameters indexed in ``model.parameters()`` order, so reference
checkpoints load and vice versa.
"""
from __future__ import annotations

import ast
import math

import torch

from hetseq_amd.ops._C import hip, stream_handle


def _as_tuple(x):
    return ast.literal_eval(x) if isinstance(x, str) else tuple(x)


_UPDATE_STREAMS: dict = {}


def update_stream(device):
    """The stream a staged update runs on (one per device, process lifetime).  A 1-GPU step uses
    the compute, weight-gradient and copy streams, so this is the fourth and gets a hardware queue
    of its own (GPU_MAX_HW_QUEUES = 4, runtime/streams.py reserve)."""
    from hetseq_amd.runtime import streams

    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _UPDATE_STREAMS.get(idx)
    if st is None:
        st = streams._new_stream(idx)
        _UPDATE_STREAMS[idx] = st
    return st


class _Optimizer(object):
    STATE_KEYS = ()

    def __init__(self, args, params, store=None):
        self.args = args
        self.param_list = [p for p in params if p.requires_grad]
        self.store = store
        self.param_groups = [dict(params=self.param_list, **self.defaults())]
        self.step_count = 0
        self._mult = None  # pending grad multiplier (float or 0-d tensor)
        self._norm_ready = False
        n = store.numel if store is not None else 0
        dev = store.device if store is not None else torch.device("cpu")
        self._state = {k: torch.zeros(n, dtype=torch.float32, device=dev) for k in self.STATE_KEYS}
        self._dev_scalars = torch.zeros(4, dtype=torch.float32, device=dev)  # [scale, norm, gmul, clip]
        self._partials = torch.zeros(1024, dtype=torch.float64, device=dev)

    # ------------------------------------------------------------ reference API
    def defaults(self):
        raise NotImplementedError

    @property
    def optimizer(self):
        return self

    @property
    def params(self):
        for p in self.param_list:
            yield p

    def get_lr(self):
        return self.param_groups[0]["lr"]

    def set_lr(self, lr):
        for g in self.param_groups:
            g["lr"] = lr

    def backward(self, loss):
        loss.backward()

    def multiply_grads(self, c):
        if self.store is None:
            for p in self.params:
                if p.grad is not None:
                    p.grad.data.mul_(c)
            return
        self._mult = c if self._mult is None else self._mult * c
        self._norm_ready = False

    def _scale_tensor(self):
        sc = self._dev_scalars[0:1]
        c = 1.0 if self._mult is None else self._mult
        if torch.is_tensor(c):
            sc.copy_(c.reshape(1).to(sc))
        else:
            sc.fill_(float(c))
        return sc

    def clip_grad_norm(self, max_norm):
        """Returns the total grad norm (after the pending multiplier) as a 0-d tensor."""
        if self.store is None:
            params = [p for p in self.params if p.grad is not None]
            if max_norm > 0:
                return torch.nn.utils.clip_grad_norm_(params, max_norm)
            return torch.sqrt(sum(p.grad.data.float().norm() ** 2 for p in params))
        self.store.flush_lazy()
        sc = self._scale_tensor()
        g = self.store.grad
        if self.store.shard is not None:  # sharded update: squares over this rank's shard, one all-reduce
            self.store.shard.grad_norm(sc, max_norm, self._dev_scalars[1:])
        elif g.is_cuda:
            hip().grad_norm(g.data_ptr(), g.numel(), self._partials.data_ptr(), sc.data_ptr(), float(max_norm),
                            self._dev_scalars[1:].data_ptr(), stream_handle())
        else:
            norm = sc[0].abs() * g.double().pow(2).sum().sqrt().float()
            clip = torch.ones((), dtype=torch.float32)
            if max_norm > 0:
                clip = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
            self._dev_scalars[1] = norm
            self._dev_scalars[2] = sc[0] * clip
            self._dev_scalars[3] = clip
        self._norm_ready = True
        return self._dev_scalars[1]

    def _grad_multiplier(self):
        """0-d device tensor multiplying every grad element in step()."""
        if not self._norm_ready:
            if self.store.grad.is_cuda:
                sc = self._scale_tensor()
                self._dev_scalars[2:3].copy_(sc)
            else:
                self._dev_scalars[2] = self._scale_tensor()[0]
        return self._dev_scalars[2:3]

    # ------------------------------------------------------------ HIP-graph support
    supports_device_hyper = False
    _hyper = None

    def enable_device_hyper(self, device):
        """Per-update hyper-parameters come from device memory (HIP-graph replay)."""
        from hetseq_amd.runtime.graphs import HostToDevice

        if not self.supports_device_hyper:
            raise NotImplementedError("%s has no device hyper-parameter path" % type(self).__name__)
        self._hyper = HostToDevice(4, torch.float32, device)

    def graph_prepare(self):
        """Host half of step() for a graph replay: count the step, publish lr / step size."""
        self.step_count += 1
        self._hyper.push(self._device_hyper_values())

    def _device_hyper_values(self):
        raise NotImplementedError

    def step(self, closure=None, launch_only=False):
        """``launch_only``: the step counter / hyper-parameters were already published by
        :meth:`graph_prepare` (graph capture); only the kernel is launched."""
        loss = closure() if closure is not None else None
        if not launch_only:
            self.step_count += 1
            if self._hyper is not None:
                self._hyper.push(self._device_hyper_values())
        if self.store is None:
            self._step_unfused()
        else:
            self.store.flush_lazy()
            gm = self._grad_multiplier()
            self.store.bump()
            if self.store.shard is not None:
                if not self.supports_staged:
                    raise NotImplementedError("%s has no sharded update" % type(self).__name__)
                self.store.shard.step(self, gm, self.staged and not torch.cuda.is_current_stream_capturing())
            elif self._staged_now():
                self._step_staged(gm)
            elif self.store.param.is_cuda:
                self._step_hip(gm)
                self.store.run_hooks()
            else:
                self._step_cpu(gm)
                self.store.run_hooks()
        self._mult = None
        self._norm_ready = False
        return loss

    # ------------------------------------------------------------ staged update
    # staged = True (the controller's choice: one GPU, eager steps, a model that declared update
    # chunks): step() runs the update chunk by chunk on update_stream(), recording a fence per chunk
    # after the chunk's update hooks; the next forward waits for each chunk just before it reads it
    # (runtime/flat.py param_ready), so the update overlaps that forward instead of preceding it.
    staged = False
    supports_staged = False

    def _staged_now(self):
        return (self.staged and self.supports_staged and self.store.chunks is not None and self.store.param.is_cuda
                and self._hyper is None and not torch.cuda.is_current_stream_capturing())

    def _step_range(self, gmul, lo, hi):
        """The update of elements [lo, hi) on the current stream (sharded and staged updates)."""
        if self.store.param.is_cuda:
            self._step_hip(gmul, lo, hi)
        else:
            self._step_cpu(gmul, lo, hi)

    def _step_staged(self, gmul):
        s = self.store
        st = update_stream(s.device)
        st.wait_stream(torch.cuda.current_stream(s.device))  # the gradients, norm and multiplier
        with torch.cuda.stream(st):
            for i, (lo, hi) in enumerate(s.chunks):
                self._step_hip(gmul, lo, hi)
                s.run_hooks(i)
                ev = torch.cuda.Event()
                ev.record(st)
                s._fences[i] = ev

    def zero_grad(self, lazy=False):
        if self.store is not None:
            self.store.zero_grad(lazy)
        else:
            for p in self.params:
                p.grad = None

    # ------------------------------------------------------------ state dict
    def _param_slices(self, key):
        buf = self._state[key]
        for p in self.param_list:
            off = self.store.offset(p)
            yield buf[off : off + p.numel()].view(p.shape)

    def consolidate(self):
        """Sharded update: gather the whole optimizer state onto every rank (collective: every rank
        calls it, before the master's state_dict())."""
        if self.store is not None and self.store.shard is not None:
            self.store.params_ready()
            self.store.shard.consolidate(self)

    def state_dict(self):
        if self.store is not None:
            self.store.params_ready()  # (a staged update may still be writing the moments)
        groups = []
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(len(self.param_list)))
            groups.append(d)
        state = {}
        if self.step_count > 0:
            slices = {k: list(self._param_slices(k)) for k in self.STATE_KEYS}
            for i in range(len(self.param_list)):
                st = {"step": self.step_count}
                for k in self.STATE_KEYS:
                    st[k] = slices[k][i]
                state[i] = st
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, state_dict, optimizer_overrides=None):
        groups = state_dict["param_groups"]
        if len(groups) != len(self.param_groups):
            raise ValueError("loaded state dict has a different number of parameter groups")
        nsaved = sum(len(g["params"]) for g in groups)
        if nsaved != len(self.param_list):
            raise ValueError("loaded state dict contains a parameter group that doesn't match the size of "
                             "optimizer's group")
        for g, sg in zip(self.param_groups, groups):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v
        st = state_dict["state"]
        if st:
            with torch.no_grad():
                for k in self.STATE_KEYS:
                    for i, sl in enumerate(self._param_slices(k)):
                        if i in st and k in st[i]:
                            sl.copy_(st[i][k].to(sl.device, sl.dtype).view(sl.shape))
            steps = [v["step"] for v in st.values() if "step" in v]
            if steps:
                s = steps[0]
                self.step_count = int(s.item() if torch.is_tensor(s) else s)
        if optimizer_overrides:
            for g in self.param_groups:
                g.update(optimizer_overrides)

    def _step_unfused(self):
        raise NotImplementedError

    def _step_hip(self, gmul):
        raise NotImplementedError

    def _step_cpu(self, gmul):
        raise NotImplementedError


class _Adam(_Optimizer):
    """fairseq "AdamW": decoupled decay applied to every parameter (Q16/Q20)."""

    STATE_KEYS = ("exp_avg", "exp_avg_sq")

    def defaults(self):
        return dict(lr=self.args.lr[0], betas=tuple(_as_tuple(self.args.adam_betas)), eps=self.args.adam_eps,
                    weight_decay=self.args.weight_decay, amsgrad=False)

    @property
    def optimizer_config(self):
        return {k: v for k, v in self.defaults().items() if k != "amsgrad"}

    supports_device_hyper = True
    supports_staged = True

    def _coeffs(self):
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        t = max(self.step_count, 1)
        step_size = g["lr"] * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        return g["lr"], b1, b2, g["eps"], g["weight_decay"], step_size

    def _device_hyper_values(self):
        lr, _, _, _, _, step_size = self._coeffs()
        return [lr, step_size, 0.0, 0.0]

    def _step_hip(self, gmul, lo=0, hi=None):
        """The fused update of elements [lo, hi) of the flat buffers (default: all)."""
        lr, b1, b2, eps, wd, step_size = self._coeffs()
        s = self.store
        hi = s.numel if hi is None else hi
        shadow = s.shadow.data_ptr() + lo * s.shadow.element_size() if s.shadow is not None else 0
        hip().adam_flat(s.param.data_ptr() + 4 * lo, s.grad.data_ptr() + 4 * lo,
                        self._state["exp_avg"].data_ptr() + 4 * lo, self._state["exp_avg_sq"].data_ptr() + 4 * lo,
                        shadow, hi - lo, gmul.data_ptr(), lr, b1, b2, eps, wd, step_size, stream_handle(),
                        self._hyper.dev.data_ptr() if self._hyper is not None else 0)

    def _step_cpu(self, gmul, lo=0, hi=None):
        lr, b1, b2, eps, wd, step_size = self._coeffs()
        s = self.store
        hi = s.numel if hi is None else hi
        with torch.no_grad():
            g = s.grad[lo:hi] * gmul
            m, v, p = self._state["exp_avg"][lo:hi], self._state["exp_avg_sq"][lo:hi], s.param[lo:hi]
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = v.sqrt().add_(eps)
            if wd != 0:
                p.add_(p, alpha=-wd * lr)
            p.addcdiv_(m, denom, value=-step_size)
            if s.shadow is not None:
                s.shadow[lo:hi].copy_(p)


class _Adadelta(_Optimizer):
    """torch Adadelta math with coupled L2 weight decay (reference: optim.py:263-304)."""

    STATE_KEYS = ("square_avg", "acc_delta")

    def defaults(self):
        return dict(lr=self.args.lr[0], rho=self.args.adadelta_rho, eps=self.args.adadelta_eps,
                    weight_decay=self.args.dadelta_weight_decay)

    @property
    def optimizer_config(self):
        return self.defaults()

    def _step_hip(self, gmul):
        g = self.param_groups[0]
        s = self.store
        shadow = s.shadow.data_ptr() if s.shadow is not None else 0
        hip().adadelta_flat(s.param.data_ptr(), s.grad.data_ptr(), self._state["square_avg"].data_ptr(),
                            self._state["acc_delta"].data_ptr(), shadow, s.numel, gmul.data_ptr(), g["lr"], g["rho"],
                            g["eps"], g["weight_decay"], stream_handle())

    def _step_cpu(self, gmul):
        grp = self.param_groups[0]
        s = self.store
        rho, eps, lr, wd = grp["rho"], grp["eps"], grp["lr"], grp["weight_decay"]
        with torch.no_grad():
            g = s.grad * gmul
            p = s.param
            if wd != 0:
                g = g.add(p, alpha=wd)
            sq, acc = self._state["square_avg"], self._state["acc_delta"]
            sq.mul_(rho).addcmul_(g, g, value=1 - rho)
            std = sq.add(eps).sqrt_()
            delta = acc.add(eps).sqrt_().div_(std).mul_(g)
            p.add_(delta, alpha=-lr)
            acc.mul_(rho).addcmul_(delta, delta, value=1 - rho)
            if s.shadow is not None:
                s.shadow.copy_(p)


class _Lamb(_Optimizer):
    """LAMB (You et al. 2019) with per-tensor trust ratios -- extension, not in the reference."""

    STATE_KEYS = ("exp_avg", "exp_avg_sq")

    def __init__(self, args, params, store=None):
        super().__init__(args, params, store)
        segs = store.segments()
        offs = [o for o, _ in segs]
        ends = [o + n for o, n in segs]
        # contiguous segment table [off_0, off_1, ..., end_last] requires adjacency; pad gaps into next segment
        table = offs + [ends[-1]]
        self._seg = torch.tensor(table, dtype=torch.int64, device=store.device)
        self._seg_norms = torch.zeros(2 * len(segs), dtype=torch.float32, device=store.device)
        self._upd = torch.zeros(store.numel, dtype=torch.float32, device=store.device)

    def defaults(self):
        return dict(lr=self.args.lr[0], betas=tuple(_as_tuple(self.args.adam_betas)), eps=self.args.adam_eps,
                    weight_decay=self.args.weight_decay)

    def _step_hip(self, gmul):
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        t = self.step_count
        s = self.store
        shadow = s.shadow.data_ptr() if s.shadow is not None else 0
        hip().lamb_flat(s.param.data_ptr(), s.grad.data_ptr(), self._state["exp_avg"].data_ptr(),
                        self._state["exp_avg_sq"].data_ptr(), self._upd.data_ptr(), shadow, self._seg.data_ptr(),
                        len(self._seg) - 1, self._seg_norms.data_ptr(), gmul.data_ptr(), g["lr"], b1, b2, g["eps"],
                        g["weight_decay"], 1 - b1 ** t, 1 - b2 ** t, stream_handle())

    def _step_cpu(self, gmul):
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        t = self.step_count
        s = self.store
        with torch.no_grad():
            grad = s.grad * gmul
            m, v = self._state["exp_avg"], self._state["exp_avg_sq"]
            m.mul_(b1).add_(grad, alpha=1 - b1)
            v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
            upd = (m / (1 - b1 ** t)) / ((v / (1 - b2 ** t)).sqrt() + g["eps"]) + g["weight_decay"] * s.param
            tab = self._seg.tolist()
            for i in range(len(tab) - 1):
                a, b = tab[i], tab[i + 1]
                pn, un = s.param[a:b].norm(), upd[a:b].norm()
                trust = (pn / un) if (pn > 0 and un > 0) else torch.tensor(1.0)
                s.param[a:b].add_(upd[a:b] * trust, alpha=-g["lr"])
            if s.shadow is not None:
                s.shadow.copy_(s.param)


def build_optimizer(args, params, store):
    name = args.optimizer
    if name == "adam":
        return _Adam(args, params, store)
    if name == "adadelta":
        return _Adadelta(args, params, store)
    if name == "lamb":
        return _Lamb(args, params, store)
    raise ValueError("unsupported optimizer - {}".format(name))


class AdamReference(torch.optim.Optimizer):
    """Per-parameter oracle of the reference Adam math (tests only)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self):
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                grad = p.grad.float()
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                b1, b2 = group["betas"]
                st["step"] += 1
                st["exp_avg"].mul_(b1).add_(grad, alpha=1 - b1)
                st["exp_avg_sq"].mul_(b2).addcmul_(grad, grad, value=1 - b2)
                denom = st["exp_avg_sq"].sqrt().add_(group["eps"])
                bc1, bc2 = 1 - b1 ** st["step"], 1 - b2 ** st["step"]
                step_size = group["lr"] * math.sqrt(bc2) / bc1
                if group["weight_decay"] != 0:
                    p.add_(p, alpha=-group["weight_decay"] * group["lr"])
                p.addcdiv_(st["exp_avg"], denom, value=-step_size)
