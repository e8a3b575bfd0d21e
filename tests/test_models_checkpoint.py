"""Model structure, heads, checkpoint format and resume (CPU)."""
import argparse
import os

import pytest
import torch

from hetseq_amd.models import bert as B


def _cfg(**kw):
    d = dict(vocab_size_or_config_json_file=200, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
             intermediate_size=128)
    d.update(kw)
    return B.BertConfig(**d)


def test_bert_base_structure_matches_reference():
    m = B.BertForPreTraining(B.BertConfig(30522))
    assert sum(p.numel() for p in m.parameters()) == 110106428
    sd = m.state_dict()
    assert len(sd) == 207
    assert sd["cls.predictions.decoder.weight"].data_ptr() == sd["bert.embeddings.word_embeddings.weight"].data_ptr()
    for k in ("bert.encoder.layer.11.attention.self.query.weight", "bert.encoder.layer.0.intermediate.dense_act.bias",
              "bert.pooler.dense_act.weight", "cls.predictions.transform.LayerNorm.weight",
              "cls.seq_relationship.bias", "cls.predictions.bias"):
        assert k in sd


def test_init_quirks():
    torch.manual_seed(0)
    m = B.BertForPreTraining(B.BertConfig(1000))
    q = m.bert.encoder.layer[0].attention.self.query
    assert abs(q.weight.std().item() - 0.02) < 2e-3 and q.bias.abs().sum() == 0
    inter = m.bert.encoder.layer[0].intermediate.dense_act
    assert inter.bias.abs().sum() > 0  # kaiming init kept (Q17)
    # deepcopy'd LinearActivation: identical across layers (reference quirk)
    assert torch.equal(inter.weight, m.bert.encoder.layer[1].intermediate.dense_act.weight)


def test_gelu_constant():
    x = torch.linspace(-4, 4, 101)
    assert torch.allclose(B.gelu(x), x * 0.5 * (1 + torch.erf(x / 1.41421)))


def test_pretraining_loss_and_heads():
    torch.manual_seed(1)
    cfg = _cfg()
    ids = torch.randint(0, 200, (3, 16))
    tt = torch.zeros_like(ids)
    mask = torch.ones_like(ids)
    lab = torch.full((3, 16), -1)
    lab[:, 2] = 5
    nsp = torch.tensor([0, 1, 0])
    m = B.BertForPreTraining(cfg)
    loss = m(ids, tt, mask, lab, nsp)
    loss.backward()
    assert loss.item() > 0 and m.bert.embeddings.word_embeddings.weight.grad is not None
    scores, rel = m(ids, tt, mask)
    assert scores.shape == (3, 16, 200) and rel.shape == (3, 2)
    assert B.BertForMaskedLM(cfg)(ids, tt, mask, lab).item() > 0
    assert B.BertForNextSentencePrediction(cfg)(ids, tt, mask, nsp).item() > 0
    assert B.BertForSequenceClassification(cfg, 3)(ids, tt, mask, torch.tensor([0, 2, 1])).item() > 0
    mc = B.BertForMultipleChoice(cfg, 2)
    assert mc(ids.view(3, 1, 16).expand(3, 2, 16), tt.view(3, 1, 16).expand(3, 2, 16),
              mask.view(3, 1, 16).expand(3, 2, 16), torch.tensor([0, 1, 1])).item() > 0
    assert B.BertForTokenClassification(cfg, 4)(ids, tt, mask, torch.randint(0, 4, (3, 16))).item() > 0
    qa = B.BertForQuestionAnswering(cfg)
    assert qa(ids, tt, mask, torch.tensor([1, 2, 3]), torch.tensor([4, 5, 6])).item() > 0


def test_checkpoint_activations_same_result():
    torch.manual_seed(2)
    m = B.BertModel(_cfg(num_hidden_layers=4)).eval()
    ids = torch.randint(0, 200, (2, 8))
    a, _ = m(ids, output_all_encoded_layers=False)
    b, _ = m(ids, output_all_encoded_layers=False, checkpoint_activations=True)
    assert torch.allclose(a, b[-1] if isinstance(b, list) else b, atol=1e-6)


def test_from_pretrained_local_dir(tmp_path):
    torch.manual_seed(3)
    cfg = _cfg()
    m = B.BertForPreTraining(cfg)
    with open(tmp_path / "bert_config.json", "w") as f:
        f.write(cfg.to_json_string())
    sd = {k.replace("LayerNorm.weight", "LayerNorm.gamma").replace("LayerNorm.bias", "LayerNorm.beta"): v
          for k, v in m.state_dict().items()}
    torch.save(sd, tmp_path / "pytorch_model.bin")
    m2 = B.BertForPreTraining.from_pretrained(str(tmp_path))
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k


def _train_cli(tmp_path, extra, data, cfg, vocab):
    from hetseq_amd.train import cli_main

    argv = ["--task", "bert", "--data", data, "--dict", vocab, "--config_file", cfg, "--max-sentences", "4",
            "--valid-subset", "test", "--cpu", "--distributed-world-size", "1", "--save-dir", str(tmp_path / "ck"),
            "--lr", "1e-3", "--log-format", "none", "--seed", "7", "--max-epoch", "3"] + extra
    return cli_main(argv)


def test_resume_is_equivalent_to_straight_run(tmp_path):
    """N updates straight == k updates, checkpoint, resume to N (fixes the reference's Q01 crash)."""
    from hetseq_amd.data.synthetic import write_bert_config, write_bert_shards, write_vocab
    from hetseq_amd.parallel import distributed_utils

    d = tmp_path / "data"
    write_bert_shards(str(d), num_shards=1, per_shard=24, seq_len=16, max_pred=3, vocab_size=200, split="train")
    write_bert_shards(str(d), num_shards=1, per_shard=4, seq_len=16, max_pred=3, vocab_size=200, split="test")
    vocab = write_vocab(str(tmp_path / "v.txt"), 200)
    cfg = write_bert_config(str(tmp_path / "c.json"), vocab_size=200, hidden_size=64, num_hidden_layers=1,
                            num_attention_heads=2, intermediate_size=128, hidden_dropout_prob=0.1)
    straight = tmp_path / "a"
    c1 = _train_cli(straight, ["--max-update", "9"], str(d), cfg, vocab)
    p_straight = c1.store.param.clone()
    resumed = tmp_path / "b"
    _train_cli(resumed, ["--max-update", "4", "--save-interval-updates", "4"], str(d), cfg, vocab)
    ck = resumed / "ck"
    assert (ck / "checkpoint_1_4.pt").exists()
    from hetseq_amd.checkpoint_utils import load_checkpoint_to_cpu

    st = load_checkpoint_to_cpu(str(ck / "checkpoint_last.pt"))
    assert set(st.keys()) == {"args", "model", "optimizer_history", "extra_state", "last_optimizer_state"}
    assert st["extra_state"]["train_iterator"]["epoch"] == 1
    assert st["optimizer_history"][-1]["optimizer_name"] == "_Adam"
    c2 = _train_cli(resumed, ["--max-update", "9"], str(d), cfg, vocab)
    assert c2.get_num_updates() == 9
    assert torch.allclose(c2.store.param, p_straight, atol=1e-6), (c2.store.param - p_straight).abs().max()
    distributed_utils.restore_output()


def test_load_reference_format_checkpoint_with_empty_extra_state(tmp_path):
    """Reference checkpoints carry extra_state == {} and a pickled Namespace (Q01/Q28)."""
    from hetseq_amd.checkpoint_utils import load_checkpoint_to_cpu

    m = B.BertForPreTraining(_cfg())
    state = {"args": argparse.Namespace(lr=[1e-4]), "model": m.state_dict(),
             "optimizer_history": [{"optimizer_name": "_Adam", "lr_scheduler_state": {"best": None},
                                    "num_updates": 3}],
             "extra_state": {}}
    torch.save(state, tmp_path / "ref.pt")
    st = load_checkpoint_to_cpu(str(tmp_path / "ref.pt"))
    assert st["optimizer_history"][0]["num_updates"] == 3 and st["extra_state"] == {}


def test_iterator_state_from_updates():
    from hetseq_amd.checkpoint_utils import iterator_state_from_updates as f

    assert f(0, 6, [1]) == {"epoch": 0, "iterations_in_epoch": 0}
    assert f(6, 6, [1]) == {"epoch": 1, "iterations_in_epoch": 0}   # epoch 1 finished
    assert f(8, 6, [1]) == {"epoch": 2, "iterations_in_epoch": 2}   # mid-epoch 2
    assert f(3, 6, [2]) == {"epoch": 1, "iterations_in_epoch": 0}   # 6 batches / uf 2 = 3 updates
    assert f(4, 7, [2]) == {"epoch": 1, "iterations_in_epoch": 0}   # ceil(7/2) = 4
    assert f(5, 6, [1, 2]) == {"epoch": 1, "iterations_in_epoch": 5}
    assert f(8, 6, [1, 2]) == {"epoch": 2, "iterations_in_epoch": 4}  # epoch 2 groups by 2


def test_resume_reference_checkpoint_keeps_epoch(tmp_path):
    """A reference-written checkpoint (extra_state == {}) resumes at the epoch its update count
    implies instead of replaying finished epochs (reference checkpoint_utils.py:115-119)."""
    from hetseq_amd.checkpoint_utils import load_checkpoint_to_cpu
    from hetseq_amd.data.synthetic import write_bert_config, write_bert_shards, write_vocab
    from hetseq_amd.parallel import distributed_utils

    d = tmp_path / "data"
    write_bert_shards(str(d), num_shards=1, per_shard=24, seq_len=16, max_pred=3, vocab_size=200, split="train")
    write_bert_shards(str(d), num_shards=1, per_shard=4, seq_len=16, max_pred=3, vocab_size=200, split="test")
    vocab = write_vocab(str(tmp_path / "v.txt"), 200)
    cfg = write_bert_config(str(tmp_path / "c.json"), vocab_size=200, hidden_size=64, num_hidden_layers=1,
                            num_attention_heads=2, intermediate_size=128)
    run = tmp_path / "r"
    c1 = _train_cli(run, ["--max-epoch", "1"], str(d), cfg, vocab)
    assert c1.get_num_updates() == 6  # 24 samples / 4 per batch
    ck = run / "ck" / "checkpoint_last.pt"
    st = load_checkpoint_to_cpu(str(ck))
    st["extra_state"] = {}  # what the reference's save_state writes (Q01)
    torch.save(st, ck)
    import shutil

    shutil.copy(ck, tmp_path / "ref_last.pt")
    c2 = _train_cli(run, ["--max-epoch", "2"], str(d), cfg, vocab)
    assert c2.get_num_updates() == 12  # epoch 2 only, not epochs 1 and 2 again
    # --reset-optimizer: the update count restarts at 0, the iterator position still comes from the
    # checkpoint's optimizer history (epoch 1 finished -> epoch 2 runs, once)
    run2 = tmp_path / "r2"
    (run2 / "ck").mkdir(parents=True)
    shutil.copy(tmp_path / "ref_last.pt", run2 / "ck" / "checkpoint_last.pt")
    c3 = _train_cli(run2, ["--max-epoch", "2", "--reset-optimizer"], str(d), cfg, vocab)
    assert c3.get_num_updates() == 6  # epoch 2's six updates, counted from 0
    st3 = load_checkpoint_to_cpu(str(run2 / "ck" / "checkpoint_last.pt"))
    assert st3["extra_state"]["train_iterator"]["epoch"] == 2
    distributed_utils.restore_output()


def test_token_classification_task_trains(tmp_path):
    """The working replacement of the reference's unreachable BertFineTuningTask (tasks.py:261-285, Q13)."""
    import argparse
    import json

    from hetseq_amd.tasks import BertTokenClassificationTask

    cfg = tmp_path / "bert_config.json"
    cfg.write_text(json.dumps(dict(vocab_size=64, hidden_size=32, num_hidden_layers=1, num_attention_heads=2,
                                   intermediate_size=64, hidden_act="gelu", hidden_dropout_prob=0.0,
                                   attention_probs_dropout_prob=0.0, max_position_embeddings=32,
                                   type_vocab_size=2, initializer_range=0.02)))
    vocab = tmp_path / "vocab.txt"
    vocab.write_text("\n".join("tok%d" % i for i in range(64)) + "\n")
    args = argparse.Namespace(config_file=str(cfg), dict=str(vocab), num_label=5)
    task = BertTokenClassificationTask.setup_task(args)
    assert len(task.dictionary) == 64
    model = task.build_model(args)

    class _Opt(object):
        def backward(self, loss):
            loss.backward()

    torch.manual_seed(0)
    ids = torch.randint(0, 64, (3, 12))
    sample = [ids, torch.zeros_like(ids), torch.ones_like(ids), torch.randint(0, 5, (3, 12))]
    loss, sample_size, log = task.train_step(sample, model, _Opt())
    # the reference's sample_size is len(sample[0][0]): the sequence length (tasks.py:164)
    assert torch.isfinite(loss) and sample_size == 12 and log["nsentences"] == 12
    assert model.classifier.weight.grad is not None and model.classifier.weight.grad.abs().sum() > 0


def test_checkpoint_names_and_pruning(tmp_path):
    """Which files a save writes (reference checkpoint_utils.py:36-55, Q07 fixed) and --keep-* pruning."""
    import argparse

    from hetseq_amd import checkpoint_utils as cu

    a = argparse.Namespace(no_epoch_checkpoints=False, save_interval=1, save_interval_updates=5,
                           no_last_checkpoints=False)
    assert cu._checkpoint_names(a, 3, 40, True, None, False) == ["checkpoint3.pt", "checkpoint_last.pt"]
    assert cu._checkpoint_names(a, 3, 40, False, None, False) == ["checkpoint_3_40.pt", "checkpoint_last.pt"]
    assert cu._checkpoint_names(a, 3, 41, False, 1.0, True) == ["checkpoint_best.pt", "checkpoint_last.pt"]
    for n in ["checkpoint1.pt", "checkpoint2.pt", "checkpoint10.pt", "checkpoint_1_5.pt", "checkpoint_1_15.pt",
              "checkpoint_last.pt"]:
        (tmp_path / n).write_text("x")
    assert [p.rsplit("/", 1)[1] for p in cu.checkpoint_paths(str(tmp_path))] == \
        ["checkpoint10.pt", "checkpoint2.pt", "checkpoint1.pt"]
    cu._prune(str(tmp_path), r"checkpoint(\d+)\.pt", 2)
    cu._prune(str(tmp_path), r"checkpoint_\d+_(\d+)\.pt", 1)
    assert sorted(p.name for p in tmp_path.iterdir()) == \
        ["checkpoint10.pt", "checkpoint2.pt", "checkpoint_1_15.pt", "checkpoint_last.pt"]
