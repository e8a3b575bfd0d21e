"""Flag parity, LR schedule, optimizer math (CPU)."""
import math
from argparse import Namespace

import pytest
import torch

from hetseq_amd import options


def _parse(extra, task="bert"):
    base = ["--task", task, "--data", "/x"]
    if task == "bert":
        base += ["--config_file", "c.json"]
    return options.parse_cli(base + extra)


def test_reference_flag_defaults():
    a = _parse([])
    exp = dict(seed=19940802, log_interval=1, log_format="simple", num_workers=0, max_tokens=None,
               max_sentences=None, required_batch_size_multiple=1, train_subset="train", valid_subset="valid",
               curriculum=0, max_pred_length=512, num_file=0, distributed_rank=0, distributed_gpus=4,
               distributed_backend="nccl", distributed_init_method=None, device_id=0, bucket_cap_mb=25,
               fast_stat_sync=False, max_epoch=0, max_update=0, clip_norm=25.0, update_freq=[1], lr=[0.25],
               min_lr=-1, use_bmuf=False, optimizer="adam", adam_betas="(0.9, 0.999)", adam_eps=1e-8,
               weight_decay=0.0, lr_scheduler="PolynomialDecayScheduler", force_anneal=None, warmup_updates=0,
               end_learning_rate=0.0, power=1.0, total_num_update=1000000, save_dir="checkpoints",
               restore_file="checkpoint_last.pt", optimizer_overrides="{}", save_interval=1,
               save_interval_updates=0, keep_interval_updates=-1, keep_last_epochs=-1, best_checkpoint_metric="loss",
               dtype="fp32")
    for k, v in exp.items():
        assert getattr(a, k) == v, k


def test_flag_aliases_and_lists():
    a = _parse(["--batch-size", "32", "--me", "3", "--mu", "9", "--wd", "0.01", "--fa", "2", "--local_rank", "1",
                "--learning-rate", "0.1,0.05", "--update-freq", "[2, 4]"])
    assert a.max_sentences == 32 and a.max_epoch == 3 and a.max_update == 9 and a.weight_decay == 0.01
    assert a.force_anneal == 2 and a.device_id == 1 and a.lr == [0.1, 0.05] and a.update_freq == [2, 4]
    assert a.max_sentences_valid == 32


def test_adadelta_flags_for_mnist():
    a = _parse(["--optimizer", "adadelta"], task="mnist")
    assert a.optimizer == "adadelta" and a.adadelta_rho == 0.9 and a.adadelta_eps == 1e-6
    assert a.dadelta_weight_decay == 0


def test_bert_requires_config_file():
    with pytest.raises(SystemExit):
        options.parse_cli(["--task", "bert", "--data", "/x"])


class _Opt:
    def __init__(self, lr):
        self.lr = lr

    def get_lr(self):
        return self.lr

    def set_lr(self, lr):
        self.lr = lr


def test_polynomial_decay_schedule():
    from hetseq_amd.optim.lr_scheduler import PolynomialDecayScheduler

    args = Namespace(lr=[1e-3], warmup_updates=10, end_learning_rate=1e-5, total_num_update=110, power=2.0,
                     force_anneal=None)
    o = _Opt(0)
    s = PolynomialDecayScheduler(args, o)
    assert s.step_update(0) == 0.0  # Q15: LR is 0 at update 0
    assert math.isclose(s.step_update(5), 5e-4)
    assert math.isclose(s.step_update(10), 1e-3)
    assert math.isclose(s.step_update(60), (1e-3 - 1e-5) * 0.5 ** 2 + 1e-5)
    assert s.step_update(110) == 1e-5 and s.step_update(500) == 1e-5
    args2 = Namespace(lr=[0.5, 0.25, 0.1], warmup_updates=0, end_learning_rate=0.0, total_num_update=10 ** 6,
                      power=1.0, force_anneal=None)
    s2 = PolynomialDecayScheduler(args2, _Opt(0))
    assert s2.step(1) == 0.25 and s2.step(7) == 0.1
    assert s2.state_dict() == {"best": None}


def _mlp():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(10, 7), torch.nn.Tanh(), torch.nn.Linear(7, 3))


def _run(opt_fn, steps=4, clip=0.5, mult=0.25):
    m = _mlp()
    opt = opt_fn(m)
    for i in range(steps):
        x = torch.randn(5, 10, generator=torch.Generator().manual_seed(i))
        opt.zero_grad()
        m(x).pow(2).sum().backward()
        opt.multiply_grads(mult)
        opt.clip_grad_norm(clip)
        opt.step()
    return m


def test_flat_adam_cpu_matches_reference_math():
    from hetseq_amd.optim.optimizers import AdamReference, _Adam
    from hetseq_amd.runtime.flat import FlatParamStore

    args = Namespace(lr=[1e-2], adam_betas="(0.9, 0.99)", adam_eps=1e-6, weight_decay=0.1)

    def fused(m):
        return _Adam(args, list(m.parameters()), FlatParamStore(m))

    m1 = _run(fused)
    m2 = _mlp()
    ref = AdamReference(m2.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-6, weight_decay=0.1)
    for i in range(4):
        x = torch.randn(5, 10, generator=torch.Generator().manual_seed(i))
        ref.zero_grad()
        m2(x).pow(2).sum().backward()
        for p in m2.parameters():
            p.grad.mul_(0.25)
        torch.nn.utils.clip_grad_norm_(list(m2.parameters()), 0.5)
        ref.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5)


def test_flat_adadelta_cpu_matches_torch():
    from hetseq_amd.optim.optimizers import _Adadelta
    from hetseq_amd.runtime.flat import FlatParamStore

    args = Namespace(lr=[1.0], adadelta_rho=0.9, adadelta_eps=1e-6, dadelta_weight_decay=0.01)
    m1 = _run(lambda m: _Adadelta(args, list(m.parameters()), FlatParamStore(m)), clip=0, mult=1.0)
    m2 = _mlp()
    ref = torch.optim.Adadelta(m2.parameters(), lr=1.0, rho=0.9, eps=1e-6, weight_decay=0.01)
    for i in range(4):
        x = torch.randn(5, 10, generator=torch.Generator().manual_seed(i))
        ref.zero_grad()
        m2(x).pow(2).sum().backward()
        ref.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5)


def test_lamb_cpu_decreases_loss():
    from hetseq_amd.optim.optimizers import _Lamb
    from hetseq_amd.runtime.flat import FlatParamStore

    args = Namespace(lr=[1e-2], adam_betas="(0.9, 0.999)", adam_eps=1e-6, weight_decay=0.01)
    m = _mlp()
    opt = _Lamb(args, list(m.parameters()), FlatParamStore(m))
    x = torch.randn(16, 10)
    losses = []
    for _ in range(20):
        opt.zero_grad()
        loss = m(x).pow(2).sum()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0]


def test_optimizer_state_dict_torch_layout_roundtrip():
    from hetseq_amd.optim.optimizers import _Adam
    from hetseq_amd.runtime.flat import FlatParamStore

    args = Namespace(lr=[1e-2], adam_betas="(0.9, 0.99)", adam_eps=1e-6, weight_decay=0.0)
    m = _run(lambda m: _Adam(args, list(m.parameters()), FlatParamStore(m)))
    # torch.optim layout, parameters indexed in model.parameters() order
    opt = _Adam(args, list(m.parameters()), FlatParamStore(m))
    m2 = _mlp()
    opt2 = _Adam(args, list(m2.parameters()), FlatParamStore(m2))
    x = torch.randn(3, 10)
    m2(x).sum().backward()
    opt2.step()
    sd = opt2.state_dict()
    assert set(sd["state"][0].keys()) == {"step", "exp_avg", "exp_avg_sq"}
    assert sd["param_groups"][0]["params"] == [0, 1, 2, 3]
    assert sd["state"][1]["exp_avg"].shape == (7,)
    opt.load_state_dict(sd, {"lr": 0.5})
    assert opt.get_lr() == 0.5 and opt.step_count == 1
    assert torch.equal(opt.state_dict()["state"][2]["exp_avg_sq"], sd["state"][2]["exp_avg_sq"])
