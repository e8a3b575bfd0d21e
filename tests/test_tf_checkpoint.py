"""TensorFlow checkpoint import without TensorFlow (reference
bert_modeling.py:43-101, 685-688).

TensorFlow is not installed and the reference ships no TF checkpoint, so the
fixtures are V2 checkpoints written by this module's own writer in the format
TF uses (SSTable index + raw data shard, uncompressed and Snappy blocks) with
Google BERT variable names: parity with TensorFlow's own files is unpinned.
"""
import json
import os

import numpy as np
import pytest
import torch


def test_snappy_copies_and_literals():
    from hetseq_amd.utils.tf_checkpoint import snappy_compress_literal, snappy_decompress

    # varint length 12, literal "abc", 1-byte-offset copy (len 9, offset 3): overlapping copy
    stream = bytes([12, (3 - 1) << 2]) + b"abc" + bytes([((9 - 4) << 2) | 1, 3])
    assert snappy_decompress(stream) == b"abcabcabcabc"
    # 2-byte-offset copy (kind 2): len 5 at offset 6
    stream = bytes([11, (6 - 1) << 2]) + b"xyzuvw" + bytes([((5 - 1) << 2) | 2, 6, 0])
    assert snappy_decompress(stream) == b"xyzuvwxyzuv"
    blob = os.urandom(70000)
    assert snappy_decompress(snappy_compress_literal(blob)) == blob


@pytest.mark.parametrize("compress", [False, True])
def test_checkpoint_roundtrip(tmp_path, compress):
    from hetseq_amd.utils.tf_checkpoint import CheckpointReader, write_checkpoint

    rng = np.random.default_rng(0)
    tensors = {"a/kernel": rng.standard_normal((7, 5)).astype(np.float32),
               "a/bias": rng.standard_normal(5).astype(np.float32),
               "global_step": np.array(1234, dtype=np.int64),
               "z/table": rng.integers(0, 100, (3, 4, 2)).astype(np.int32),
               "h": rng.standard_normal(6).astype(np.float16)}
    write_checkpoint(str(tmp_path / "model.ckpt"), tensors, compress=compress)
    r = CheckpointReader(str(tmp_path / "model.ckpt.index"))
    assert [n for n, _ in r.list_variables()] == sorted(tensors)
    for k, v in tensors.items():
        got = r.get_tensor(k)
        assert got.dtype == v.dtype and got.shape == v.shape and np.array_equal(got, v), k


def _google_names(model):
    """The Google BERT checkpoint layout of a BertForPreTraining (TF kernels are [in, out])."""
    out = {}
    for k, v in model.state_dict().items():
        if k == "cls.predictions.decoder.weight":
            continue  # tied to the word embeddings; not stored by TF
        a = v.detach().numpy().copy()
        parts = k.split(".")
        name = []
        i = 0
        while i < len(parts):
            p = parts[i]
            if p == "layer" and i + 1 < len(parts) and parts[i + 1].isdigit():
                name.append("layer_" + parts[i + 1])
                i += 2
                continue
            name.append(p)
            i += 1
        leaf = name[-1]
        if name[-2].endswith("_embeddings") and leaf == "weight":
            name = name[:-1]
        elif name[:2] == ["cls", "seq_relationship"]:
            name[-1] = "output_weights" if leaf == "weight" else "output_bias"
        elif name[:2] == ["cls", "predictions"] and len(name) == 3 and leaf == "bias":
            name[-1] = "output_bias"
        elif "LayerNorm" in name:
            name[-1] = "gamma" if leaf == "weight" else "beta"
        elif leaf == "weight":
            name[-1] = "kernel"
            a = a.T.copy()
        out["/".join(name)] = a
    return out


def test_bert_from_tf_checkpoint(tmp_path):
    from hetseq_amd.models.bert import BertConfig, BertForPreTraining
    from hetseq_amd.utils.tf_checkpoint import write_checkpoint

    cfg = dict(vocab_size=120, hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64,
               hidden_act="gelu", hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1,
               max_position_embeddings=64, type_vocab_size=2, initializer_range=0.02)
    torch.manual_seed(3)
    src = BertForPreTraining(BertConfig(vocab_size_or_config_json_file=120, **{k: v for k, v in cfg.items()
                                                                               if k != "vocab_size"}))
    tensors = _google_names(src)
    assert "bert/encoder/layer_1/attention/self/query/kernel" in tensors
    assert "cls/predictions/output_bias" in tensors and "cls/seq_relationship/output_weights" in tensors
    # optimizer slots and the step counter are in real checkpoints; the loader skips them
    tensors["bert/encoder/layer_0/output/dense/kernel/adam_m"] = np.zeros((64, 32), np.float32)
    tensors["global_step"] = np.array(7, dtype=np.int64)
    d = tmp_path / "tfbert"
    d.mkdir()
    write_checkpoint(str(d / "bert_model.ckpt"), tensors, compress=True)
    with open(d / "bert_config.json", "w") as f:
        json.dump(cfg, f)
    torch.manual_seed(99)
    dst = BertForPreTraining.from_pretrained(str(d), from_tf=True)
    ref, got = src.state_dict(), dst.state_dict()
    for k in ref:
        assert torch.equal(ref[k], got[k]), k
    # the tied decoder still shares the (loaded) word-embedding storage
    assert dst.cls.predictions.decoder.weight.data_ptr() == dst.bert.embeddings.word_embeddings.weight.data_ptr()
