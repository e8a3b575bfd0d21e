"""--hip-graph: the captured-and-replayed update must train exactly like the eager one
(same dropout stream through the device seed, same lr / bias correction through the
device hyper-parameters).  Single GPU, tiny BERT, synthetic shards."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(tmp_path, hip_graph, steps, dtype="fp32"):
    from hetseq_amd import options
    from hetseq_amd.controller import Controller
    from hetseq_amd.data.synthetic import write_bert_config, write_bert_shards, write_vocab
    from hetseq_amd.runtime import rng
    from hetseq_amd.tasks import LanguageModelingTask

    V = 1000
    d = str(tmp_path / ("g%d%s" % (int(hip_graph), dtype)))
    write_bert_shards(os.path.join(d, "data"), num_shards=1, per_shard=16 * (steps + 2), seq_len=128, max_pred=20,
                      vocab_size=V, seed=5, split="train")
    write_vocab(os.path.join(d, "vocab.txt"), V)
    cfg = write_bert_config(os.path.join(d, "cfg.json"), vocab_size=V, hidden_size=256, num_hidden_layers=2,
                            num_attention_heads=4, intermediate_size=1024)
    argv = ["--task", "bert", "--data", os.path.join(d, "data"), "--dict", os.path.join(d, "vocab.txt"),
            "--config_file", cfg, "--max-sentences", "16", "--lr", "1e-3", "--warmup-updates", "4",
            "--max-update", "100", "--fast-stat-sync", "--clip-norm", "1.0", "--dtype", dtype,
            "--distributed-world-size", "1", "--log-format", "none"] + (["--hip-graph"] if hip_graph else [])
    args = options.parse_cli(argv)
    torch.manual_seed(args.seed)
    task = LanguageModelingTask.setup_task(args)
    model = task.build_model(args)
    ctl = Controller(args, task, model)
    task.load_dataset("train")
    task.prepare_model_for_data(ctl.get_model(), "train")
    itr = task.get_batch_iterator(task.dataset("train"), max_sentences=16, seed=args.seed, num_workers=1, epoch=0,
                                  device=ctl.device).next_epoch_itr(shuffle=False)
    losses = []
    for _, s in zip(range(steps), itr):
        out = ctl.train_step([s])
        losses.append(float(out["loss"]))
    params = ctl.store.param.clone()
    rng.disable_device_seed()
    return losses, params, ctl


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_graph_replay_matches_eager(cuda, tmp_path, dtype):
    steps = 8  # 3 eager warm-up updates, capture on the 4th, 4 replays
    l_eager, p_eager, _ = _run(tmp_path, False, steps, dtype)
    l_graph, p_graph, ctl = _run(tmp_path, True, steps, dtype)
    assert ctl._graph is not None and ctl._graph.graph is not None
    assert ctl.optimizer.step_count == steps
    for a, b in zip(l_eager, l_graph):
        assert abs(a - b) <= 1e-5 * abs(a) + 1e-6, (l_eager, l_graph)
    err = (p_eager - p_graph).abs().max().item()
    assert err <= 1e-5 * p_eager.abs().max().item(), err


def test_controller_leaves_tunableop_off(cuda, tmp_path):
    """Building and stepping a default Controller must not switch on process-global TunableOp
    (the library-GEMM table is an entry-point decision: runtime.gemm_tuning.configure)."""
    import torch.cuda.tunable as tn

    _run(tmp_path, False, 1)
    assert not tn.is_enabled()
    assert not tn.tuning_is_enabled()
