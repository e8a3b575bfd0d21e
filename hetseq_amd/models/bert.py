"""BERT model family (reference: bert_modeling.py).

What must match the reference, and why:
  * the module tree and parameter names -- 207 state-dict keys for BERT-base,
    tied MLM decoder -- because checkpoints and ``from_pretrained`` archives
    are exchanged with it (reference :292-888);
  * the numerics of the pre-training forward: post-LN encoder, separate
    Q/K/V projections, additive (1 - mask) * -10000 attention mask (Q27),
    dropout on the attention probabilities, erf-GELU with the 1.41421
    constant (Q18), TF-style LayerNorm with eps 1e-12, MLM CE(ignore -1) +
    NSP CE as the returned loss (reference :875-888);
  * the initialisation quirks: N(0, 0.02) for Linear / Embedding weights via
    ``init_bert_weights`` (applied by BertModel and again by each heads
    model), while ``LinearActivation`` keeps its uniform(+-1/sqrt(fan_in))
    weight AND bias and is deep-copied across encoder layers (Q17).

Two execution paths share the modules:
  * fused (GPU): ``FusedEmbedding`` -> L x ``FusedBertLayer`` -> the fused
    pre-training heads (sparse MLM + pooler/NSP) over the gfx950 HIP kernels
    in hetseq_amd/ops/bert_ops.py, fp32 or bf16 compute;
  * torch-op oracle (CPU, ``--no-fused``, fine-tuning heads): plain PyTorch,
    the numerical reference the kernel tests compare against.
"""
from __future__ import annotations

import copy
import json
import logging
import math
import os
import shutil
import tarfile
import tempfile

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.parameter import Parameter
from torch.utils import checkpoint

logger = logging.getLogger(__name__)

TF_WEIGHTS_NAME = "model.ckpt"
CONFIG_NAME = "bert_config.json"
WEIGHTS_NAME = "pytorch_model.bin"
FUSED_HIDDEN = (256, 512, 768, 1024, 1536, 2048)  # widths the LayerNorm / embedding kernels serve


# ----------------------------------------------------------------- activations (reference :104-130)
_ERF_DIV = 1.41421  # the reference's constant, not sqrt(2) (Q18)


def f_gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x / _ERF_DIV))


gelu = f_gelu


def bias_gelu(bias, y):
    return f_gelu(y + bias)


def bias_tanh(bias, y):
    return torch.tanh(y + bias)


def swish(x):
    return torch.sigmoid(x) * x


ACT2FN = {"gelu": gelu, "relu": F.relu, "swish": swish, "tanh": torch.tanh}


def _fused_ok(t):
    from hetseq_amd.ops._C import use_fused

    return use_fused(t)


def _cw(w, x):
    """``w`` in the compute dtype of ``x`` (autograd-transparent cast)."""
    return w if w.dtype == x.dtype else w.to(x.dtype)


class LinearActivation(nn.Module):
    """act(x @ W^T + b) with the bias added by the activation step (reference :132-177).

    Parameters are initialised like ``torch.nn.Linear`` (uniform, bound 1/sqrt(fan_in) for weight
    and bias), and ``init_bert_weights`` does not touch this class -- the reference quirk kept."""

    def __init__(self, in_features, out_features, act="gelu", bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.act = act
        self.weight = Parameter(torch.empty(out_features, in_features))
        if bias:
            self.bias = Parameter(torch.empty(out_features))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    @property
    def fused_gelu(self):
        return self.act == "gelu" and self.bias is not None

    def reset_parameters(self):
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            lim = self.in_features ** -0.5
            nn.init.uniform_(self.bias, -lim, lim)

    def forward(self, x):
        y = F.linear(x, _cw(self.weight, x))
        if self.bias is None:
            return (ACT2FN[self.act] if isinstance(self.act, str) else self.act)(y)
        if self.act == "gelu":
            if _fused_ok(x) and x.dim() == 2 and self.out_features % 4 == 0:
                from hetseq_amd.ops.bert_ops import bias_gelu as hip_bias_gelu

                return hip_bias_gelu(y, self.bias)
            return bias_gelu(self.bias, y)
        if self.act == "tanh":
            return bias_tanh(self.bias, y)
        fn = ACT2FN[self.act] if isinstance(self.act, str) else self.act
        return fn(y + self.bias)

    def extra_repr(self):
        return "in_features=%d, out_features=%d, bias=%s" % (self.in_features, self.out_features,
                                                               self.bias is not None)


# ----------------------------------------------------------------- configuration (reference :180-266)
# (JSON key, default) -- the reference's config schema, in its positional order
_CONFIG_FIELDS = (("hidden_size", 768), ("num_hidden_layers", 12), ("num_attention_heads", 12),
                  ("intermediate_size", 3072), ("hidden_act", "gelu"), ("hidden_dropout_prob", 0.1),
                  ("attention_probs_dropout_prob", 0.1), ("max_position_embeddings", 512),
                  ("type_vocab_size", 2), ("initializer_range", 0.02))


def _read_json(path):
    with open(path, "r", encoding="utf-8") as f:
        return json.load(f)


class BertConfig(object):
    """BERT hyper-parameters.  ``BertConfig(vocab_size, **fields)`` or ``BertConfig(path.json)``;
    the JSON keys are those of Google's ``bert_config.json``."""

    def __init__(self, vocab_size_or_config_json_file, *args, **kwargs):
        src = vocab_size_or_config_json_file
        if isinstance(src, str):
            self.__dict__.update(_read_json(src))
            return
        if not isinstance(src, int):
            raise ValueError("First argument must be either a vocabulary size (int) or the path to a pretrained "
                             "model config file (str)")
        names = [n for n, _ in _CONFIG_FIELDS]
        if len(args) > len(names):
            raise TypeError("BertConfig takes at most %d positional fields" % len(names))
        unknown = sorted(set(kwargs) - set(names))
        if unknown:
            raise TypeError("unknown BertConfig field(s): %s" % ", ".join(unknown))
        fields = dict(_CONFIG_FIELDS)
        fields.update(zip(names, args))
        fields.update(kwargs)
        self.vocab_size = src
        self.__dict__.update(fields)

    @classmethod
    def from_dict(cls, json_object):
        cfg = cls.__new__(cls)
        cfg.__dict__.update(copy.deepcopy(dict(json_object)))
        return cfg

    @classmethod
    def from_json_file(cls, json_file):
        return cls.from_dict(_read_json(json_file))

    def to_dict(self):
        return copy.deepcopy(self.__dict__)

    def to_json_string(self):
        return json.dumps(self.to_dict(), indent=2, sort_keys=True) + "\n"

    def __repr__(self):
        return self.to_json_string()


class BertLayerNorm(nn.Module):
    """TF-style LayerNorm: (x - mean) / sqrt(biased var + eps) * weight + bias (reference :277-289)."""

    def __init__(self, hidden_size, eps=1e-12):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size))
        self.bias = nn.Parameter(torch.zeros(hidden_size))
        self.variance_epsilon = eps

    def forward(self, x):
        if _fused_ok(x) and x.shape[-1] in FUSED_HIDDEN:
            from hetseq_amd.ops.bert_ops import layer_norm

            flat = x.reshape(-1, x.shape[-1]).contiguous()
            return layer_norm(flat, self.weight, self.bias, self.variance_epsilon).view(x.shape)
        centered = x - x.mean(-1, keepdim=True)
        inv = torch.rsqrt(centered.pow(2).mean(-1, keepdim=True) + self.variance_epsilon)
        return centered * inv * self.weight + self.bias


# ----------------------------------------------------------------- encoder modules
class BertEmbeddings(nn.Module):
    """word + position + token-type embeddings -> LayerNorm -> dropout (reference :292-320)."""

    def __init__(self, config):
        super().__init__()
        H = config.hidden_size
        self.word_embeddings = nn.Embedding(config.vocab_size, H)
        self.position_embeddings = nn.Embedding(config.max_position_embeddings, H)
        self.token_type_embeddings = nn.Embedding(config.type_vocab_size, H)
        self.LayerNorm = BertLayerNorm(H, eps=1e-12)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, input_ids, token_type_ids=None):
        S = input_ids.shape[1]
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        pos = self.position_embeddings.weight[:S].unsqueeze(0)  # positions 0..S-1, broadcast over B
        summed = self.word_embeddings(input_ids) + pos + self.token_type_embeddings(token_type_ids)
        return self.dropout(self.LayerNorm(summed))

    def fused(self, input_ids, token_type_ids, out_dtype, amax=None):
        from hetseq_amd.ops.bert_ops import FusedEmbedding

        p = self.dropout.p if self.training else 0.0
        params = [self.word_embeddings.weight, self.position_embeddings.weight, self.token_type_embeddings.weight,
                  self.LayerNorm.weight, self.LayerNorm.bias]
        store = getattr(self, "_hs_store", None)
        sink = {"views": lambda: [store.grad_view(q) for q in params]} if store is not None else None
        return FusedEmbedding.apply(input_ids, token_type_ids, *params, p, self.LayerNorm.variance_epsilon,
                                    out_dtype, sink, amax)


class BertSelfAttention(nn.Module):
    """Multi-head scaled dot-product attention with separate Q/K/V projections (reference :323-377)."""

    def __init__(self, config):
        super().__init__()
        H, nh = config.hidden_size, config.num_attention_heads
        if H % nh:
            raise ValueError("The hidden size (%d) is not a multiple of the number of attention heads (%d)" % (H, nh))
        self.num_attention_heads = nh
        self.attention_head_size = H // nh
        self.all_head_size = nh * self.attention_head_size
        self.query = nn.Linear(H, self.all_head_size)
        self.key = nn.Linear(H, self.all_head_size)
        self.value = nn.Linear(H, self.all_head_size)
        self.dropout = nn.Dropout(config.attention_probs_dropout_prob)
        # Q/K/V weights (and biases) adjacent in the flat store -> one [3H, H] GEMM operand
        self._flat_groups = [[self.query.weight, self.key.weight, self.value.weight],
                             [self.query.bias, self.key.bias, self.value.bias]]

    def _heads(self, t):
        """[B, S, nh * dh] -> [B, nh, S, dh]"""
        B, S, _ = t.shape
        return t.reshape(B, S, self.num_attention_heads, self.attention_head_size).transpose(1, 2)

    def forward(self, hidden_states, attention_mask):
        q, k, v = (self._heads(proj(hidden_states)) for proj in (self.query, self.key, self.value))
        scores = q.matmul(k.transpose(-1, -2)) / math.sqrt(self.attention_head_size) + attention_mask
        probs = self.dropout(torch.softmax(scores, dim=-1))
        ctx = probs.matmul(v).transpose(1, 2)
        return ctx.reshape(ctx.shape[0], ctx.shape[1], self.all_head_size)


class _DenseDropoutAddNorm(nn.Module):
    """LayerNorm(dropout(dense(x)) + residual): the shared shape of BertSelfOutput (reference
    :380-391) and BertOutput (:416-427)."""

    def __init__(self, in_features, config):
        super().__init__()
        self.dense = nn.Linear(in_features, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=1e-12)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, hidden_states, input_tensor):
        return self.LayerNorm(input_tensor + self.dropout(self.dense(hidden_states)))


class BertSelfOutput(_DenseDropoutAddNorm):
    def __init__(self, config):
        super().__init__(config.hidden_size, config)


class BertOutput(_DenseDropoutAddNorm):
    def __init__(self, config):
        super().__init__(config.intermediate_size, config)


class BertAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.self = BertSelfAttention(config)
        self.output = BertSelfOutput(config)

    def forward(self, input_tensor, attention_mask):
        return self.output(self.self(input_tensor, attention_mask), input_tensor)


class BertIntermediate(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense_act = LinearActivation(config.hidden_size, config.intermediate_size, act=config.hidden_act)

    def forward(self, hidden_states):
        return self.dense_act(hidden_states)


class BertLayer(nn.Module):
    """Post-LN transformer block (reference :430-441) plus the fused-kernel plumbing."""

    def __init__(self, config):
        super().__init__()
        self.attention = BertAttention(config)
        self.intermediate = BertIntermediate(config)
        self.output = BertOutput(config)

    def forward(self, hidden_states, attention_mask):
        attended = self.attention(hidden_states, attention_mask)
        return self.output(self.intermediate(attended), attended)

    # ------------------------------------------------------------- fused path
    def fused_params(self):
        """The 16 parameters in reference order (q.w, q.b, k.w, k.b, v.w, v.b, o.w, o.b, ln1.w,
        ln1.b, i.w, i.b, out.w, out.b, ln2.w, ln2.b); parameter objects never change identity."""
        cached = self.__dict__.get("_hs_pcache")
        if cached is None:
            sa, so, o = self.attention.self, self.attention.output, self.output
            mods = (sa.query, sa.key, sa.value, so.dense, so.LayerNorm, self.intermediate.dense_act, o.dense,
                    o.LayerNorm)
            cached = [t for m in mods for t in (m.weight, m.bias)]
            self.__dict__["_hs_pcache"] = cached
        return cached

    def _weights(self):
        """Kernel-side weight views.  With a flat store they are fixed views into its buffers
        (parameters are updated in place), so they are built once and cached.  ``W.h3p``: the GEMM
        weights' h3p planes this forward's encoder refreshed (None: the layer runs another engine)."""
        cached = getattr(self, "_hs_wcache", None)
        if cached is None:
            cached = self._build_weights()
            if getattr(self, "_hs_store", None) is not None:
                self._hs_wcache = cached
        cached.h3p = self.__dict__.get("_hs_h3p_cur")
        return cached

    def _build_weights(self):
        from hetseq_amd.ops.bert_ops import LayerWeights

        store = getattr(self, "_hs_store", None)
        bf16 = getattr(self, "_hs_dtype", torch.float32) == torch.bfloat16
        sa, ao, o = self.attention.self, self.attention.output, self.output
        H = sa.query.weight.shape[1]
        W = LayerWeights()

        def cw(p):  # GEMM weight in compute dtype
            if not bf16:
                return p.detach()
            if store is not None:
                return store.shadow_view(p)
            return p.detach().to(torch.bfloat16)

        qkv = [sa.query.weight, sa.key.weight, sa.value.weight]
        wqkv = store.combined(qkv, (3 * sa.all_head_size, H), shadow=bf16) if store is not None else None
        if wqkv is None:
            wqkv = torch.cat([cw(p) for p in qkv], 0)
        bqkv = store.combined([sa.query.bias, sa.key.bias, sa.value.bias], (3 * sa.all_head_size,)) \
            if store is not None else None
        if bqkv is None:
            bqkv = torch.cat([sa.query.bias.detach(), sa.key.bias.detach(), sa.value.bias.detach()])
        W.wqkv, W.bqkv = wqkv, bqkv
        W.wo, W.bo = cw(ao.dense.weight), ao.dense.bias.detach()
        W.g1, W.b1 = ao.LayerNorm.weight.detach(), ao.LayerNorm.bias.detach()
        W.w1, W.bi = cw(self.intermediate.dense_act.weight), self.intermediate.dense_act.bias.detach()
        W.w2, W.b2 = cw(o.dense.weight), o.dense.bias.detach()
        W.g2, W.bb2 = o.LayerNorm.weight.detach(), o.LayerNorm.bias.detach()
        return W

    def grad_groups(self):
        """This layer's parameters in the order the fused backward completes their gradients (FFN-out
        + LN2, FFN-in, attention output + LN1, QKV): what the data-parallel engine may reduce one
        group at a time (parallel/ddp.py early buckets)."""
        sa, ao, o = self.attention.self, self.attention.output, self.output
        return [[o.dense.weight, o.dense.bias, o.LayerNorm.weight, o.LayerNorm.bias],
                [self.intermediate.dense_act.weight, self.intermediate.dense_act.bias],
                [ao.dense.weight, ao.dense.bias, ao.LayerNorm.weight, ao.LayerNorm.bias],
                [sa.query.weight, sa.key.weight, sa.value.weight, sa.query.bias, sa.key.bias, sa.value.bias]]

    def fused_ok(self, x, S):
        sa = self.attention.self
        H = sa.query.weight.shape[1]
        return (sa.attention_head_size == 64 and H in FUSED_HIDDEN and S % 32 == 0
                and self.intermediate.dense_act.fused_gelu and self.intermediate.dense_act.out_features % 4 == 0)

    def fused(self, x2d, mask_i64, B, S, recompute=False, amax=None):
        """``amax``: this layer's bert_ops.LayerAmax (h3 GEMM engine operand scales) or None."""
        from hetseq_amd.ops.bert_ops import FusedBertLayer
        from hetseq_amd.runtime import rng

        p_h = self.output.dropout.p if self.training else 0.0
        p_a = self.attention.self.dropout.p if self.training else 0.0
        seeds = tuple(rng.fork() if p > 0 else (0, 0) for p in (p_a, p_h, p_h))
        cfg = (B, S, self.attention.self.num_attention_heads, p_h, p_a, self.output.LayerNorm.variance_epsilon, seeds)
        meta = {"weights": self._weights, "cfg": cfg, "recompute": recompute, "amax": amax}
        store = getattr(self, "_hs_store", None)
        if store is not None:
            meta["grad_sink"] = self._grad_views
            meta["store"] = store
            early = self.__dict__.get("_hs_early")  # (parallel/ddp.py) per-group readiness of this layer
            if early is not None:
                meta["early"] = early
            if x2d.requires_grad:
                # gradients go straight into the store: no parameter inputs (no AccumulateGrad nodes,
                # no per-parameter hooks); the backward reports the layer's parameters ready at its end
                ready = getattr(store, "ready_cb", None)
                if ready is not None:
                    params = self.fused_params()
                    meta["ready"] = lambda: ready(params)
                return FusedBertLayer.apply(x2d, mask_i64, meta)
        return FusedBertLayer.apply(x2d, mask_i64, meta, *self.fused_params())

    def _grad_views(self):
        """fp32 views of this layer's gradients inside the flat store (accumulated in place)."""
        cached = getattr(self, "_hs_gcache", None)
        if cached is not None and cached[0] is self._hs_store:
            return cached[1]
        G = self._build_grad_views()
        self._hs_gcache = (self._hs_store, G)
        return G

    def _build_grad_views(self):
        from hetseq_amd.ops.bert_ops import LayerWeights

        store = self._hs_store
        sa, ao, o = self.attention.self, self.attention.output, self.output
        H = sa.query.weight.shape[1]
        g = LayerWeights()
        g.wqkv = store.combined_grad([sa.query.weight, sa.key.weight, sa.value.weight], (3 * sa.all_head_size, H))
        g.bqkv = store.combined_grad([sa.query.bias, sa.key.bias, sa.value.bias], (3 * sa.all_head_size,))
        assert g.wqkv is not None and g.bqkv is not None, "Q/K/V parameters are not adjacent in the flat store"
        gv = store.grad_view
        g.wo, g.bo = gv(ao.dense.weight), gv(ao.dense.bias)
        g.g1, g.b1 = gv(ao.LayerNorm.weight), gv(ao.LayerNorm.bias)
        g.w1, g.bi = gv(self.intermediate.dense_act.weight), gv(self.intermediate.dense_act.bias)
        g.w2, g.b2 = gv(o.dense.weight), gv(o.dense.bias)
        g.g2, g.bb2 = gv(o.LayerNorm.weight), gv(o.LayerNorm.bias)
        store.cover(g.wqkv, g.wo, g.w1, g.w2)  # the fused backward overwrites these (lazy zero_grad)
        return g


class BertEncoder(nn.Module):
    """L identical (deep-copied) layers; optional activation checkpointing over ceil(sqrt(L))-layer
    segments (reference :444-487)."""

    def __init__(self, config):
        super().__init__()
        proto = BertLayer(config)
        self.layer = nn.ModuleList([copy.deepcopy(proto) for _ in range(config.num_hidden_layers)])

    def _run(self, first, last):
        def segment(h, mask):
            for blk in self.layer[first:last]:
                h = blk(h, mask)
            return h

        return segment

    def forward(self, hidden_states, attention_mask, output_all_encoded_layers=True, checkpoint_activations=False):
        if checkpoint_activations:
            L = len(self.layer)
            step = math.ceil(math.sqrt(L))
            for first in range(0, L, step):
                hidden_states = checkpoint.checkpoint(self._run(first, first + step), hidden_states,
                                                      attention_mask * 1, use_reentrant=False)
            return [hidden_states]
        outs = []
        for blk in self.layer:
            hidden_states = blk(hidden_states, attention_mask)
            outs.append(hidden_states)
        return outs if output_all_encoded_layers else outs[-1:]


# ----------------------------------------------------------------- heads (reference :506-581)
class BertPooler(nn.Module):
    """tanh(dense(first token))."""

    def __init__(self, config):
        super().__init__()
        self.dense_act = LinearActivation(config.hidden_size, config.hidden_size, act="tanh")

    def forward(self, hidden_states):
        return self.dense_act(hidden_states[:, 0])


class BertPredictionHeadTransform(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense_act = LinearActivation(config.hidden_size, config.hidden_size, act=config.hidden_act)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=1e-12)

    def forward(self, hidden_states):
        return self.LayerNorm(self.dense_act(hidden_states))


class BertLMPredictionHead(nn.Module):
    """transform -> decoder tied to the word embeddings (no bias of its own) + a separate bias."""

    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        V, H = bert_model_embedding_weights.shape
        self.transform = BertPredictionHeadTransform(config)
        self.decoder = nn.Linear(H, V, bias=False)
        self.decoder.weight = bert_model_embedding_weights
        self.bias = nn.Parameter(torch.zeros(V))

    def forward(self, hidden_states):
        from hetseq_amd.runtime.profiling import range_pop, range_push

        h = self.transform(hidden_states)
        range_push("decoder")
        try:
            return F.linear(h, self.decoder.weight, self.bias)
        finally:
            range_pop()


class BertOnlyMLMHead(nn.Module):
    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        self.predictions = BertLMPredictionHead(config, bert_model_embedding_weights)

    def forward(self, sequence_output):
        return self.predictions(sequence_output)


class BertOnlyNSPHead(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.seq_relationship = nn.Linear(config.hidden_size, 2)

    def forward(self, pooled_output):
        return self.seq_relationship(pooled_output)


class BertPreTrainingHeads(nn.Module):
    """MLM prediction head + NSP classifier (registered in that order: it fixes the parameter
    order, hence the optimizer-state indices of reference checkpoints)."""

    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        self.predictions = BertLMPredictionHead(config, bert_model_embedding_weights)
        self.seq_relationship = nn.Linear(config.hidden_size, 2)

    def forward(self, sequence_output, pooled_output):
        return self.predictions(sequence_output), self.seq_relationship(pooled_output)


# ----------------------------------------------------------------- checkpoint import
def _pretrained_key(name):
    """Names of pre-PyTorch-era BERT archives (LayerNorm gamma/beta) -> this module tree."""
    return name.replace("gamma", "weight").replace("beta", "bias")


def load_pretrained_state(model, state_dict):
    """Load an archive state dict into ``model`` (non-strict: heads absent from the archive keep
    their fresh init).  Renames gamma/beta, and drops a leading ``bert.`` when ``model`` is the bare
    encoder.  Shape mismatches raise; missing / unused keys are logged (reference :690-733)."""
    remapped = {_pretrained_key(k): v for k, v in state_dict.items()}
    if not hasattr(model, "bert") and any(k.startswith("bert.") for k in remapped):
        remapped = {k[len("bert."):] if k.startswith("bert.") else k: v for k, v in remapped.items()}
    result = model.load_state_dict(remapped, strict=False)
    if result.missing_keys:
        logger.info("Weights of %s not initialized from pretrained model: %s", type(model).__name__,
                    result.missing_keys)
    if result.unexpected_keys:
        logger.info("Weights from pretrained model not used in %s: %s", type(model).__name__,
                    result.unexpected_keys)
    return model


class BertPreTrainedModel(nn.Module):
    """Weight init, runtime plumbing (flat store, compute dtype) and local ``from_pretrained``."""

    def __init__(self, config, *inputs, **kwargs):
        super().__init__()
        if not isinstance(config, BertConfig):
            raise ValueError("Parameter config in `{}(config)` should be an instance of class `BertConfig`."
                             .format(type(self).__name__))
        self.config = config

    def init_bert_weights(self, module):
        """N(0, initializer_range) for Linear / Embedding weights, zero Linear biases, identity
        LayerNorm; LinearActivation is deliberately not matched (reference :599-610)."""
        std = self.config.initializer_range
        if isinstance(module, BertLayerNorm):
            nn.init.ones_(module.weight)
            nn.init.zeros_(module.bias)
            return
        if isinstance(module, (nn.Linear, nn.Embedding)):
            module.weight.data.normal_(0.0, std)
        if isinstance(module, nn.Linear) and module.bias is not None:
            nn.init.zeros_(module.bias)

    # --- runtime plumbing (flat store / compute dtype / fused switch)
    def attach_store(self, store, compute_dtype=torch.float32):
        for m in self.modules():
            m._hs_store = store
            m._hs_dtype = compute_dtype
            m._hs_wcache = None
        self._compute_dtype = compute_dtype
        groups = self.update_groups()
        if groups is not None and store is not None:
            store.set_chunks(groups)

    def update_groups(self):
        """Parameter groups in the order the fused forward first reads them (the staged update's
        chunks, runtime/flat.py set_chunks); None: no chunk-aware forward."""
        return None

    def set_compute_dtype(self, dtype):
        for m in self.modules():
            m._hs_dtype = dtype
            m._hs_wcache = None
        self._compute_dtype = dtype

    @property
    def compute_dtype(self):
        return getattr(self, "_hs_dtype", torch.float32)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, state_dict=None, cache_dir=None, from_tf=False, *inputs,
                        **kwargs):
        """Build from a local directory or ``.tar.gz`` archive (bert_config.json + pytorch_model.bin,
        or a TF checkpoint with ``from_tf``).  There is no network: remote names resolve only through
        :func:`hetseq_amd.utils.file_utils.cached_path`'s cache.  Weights load with
        ``weights_only=True``; TF checkpoints are read without TensorFlow."""
        from hetseq_amd.utils.file_utils import cached_path

        resolved = cached_path(pretrained_model_name_or_path, cache_dir=cache_dir)
        unpacked = None
        if not (os.path.isdir(resolved) or from_tf):
            unpacked = tempfile.mkdtemp()
            with tarfile.open(resolved, "r:gz") as archive:
                archive.extractall(unpacked, filter="data")
        root = unpacked or resolved
        try:
            model = cls(BertConfig.from_json_file(os.path.join(root, CONFIG_NAME)), *inputs, **kwargs)
            if from_tf:
                from hetseq_amd.utils.tf_checkpoint import load_tf_weights_in_bert

                prefix = os.path.join(root, TF_WEIGHTS_NAME)
                if not os.path.exists(prefix + ".index") and os.path.exists(os.path.join(root,
                                                                                        "bert_model.ckpt.index")):
                    prefix = os.path.join(root, "bert_model.ckpt")  # Google's release name
                return load_tf_weights_in_bert(model, prefix)
            if state_dict is None:
                state_dict = torch.load(os.path.join(root, WEIGHTS_NAME), map_location="cpu", weights_only=True)
        finally:
            if unpacked:
                shutil.rmtree(unpacked, ignore_errors=True)
        return load_pretrained_state(model, state_dict)


class BertModel(BertPreTrainedModel):
    """Embeddings + encoder + pooler; returns (encoded layers, pooled first token)."""

    def __init__(self, config):
        super().__init__(config)
        self.embeddings = BertEmbeddings(config)
        self.encoder = BertEncoder(config)
        self.pooler = BertPooler(config)
        self.apply(self.init_bert_weights)

    def _can_fuse(self, input_ids):
        if not _fused_ok(input_ids) or getattr(self, "_hs_disable_fused", False):
            return False
        S = input_ids.shape[-1]
        return self.config.hidden_size in FUSED_HIDDEN and all(blk.fused_ok(None, S) for blk in self.encoder.layer)

    @staticmethod
    def additive_mask(attention_mask, dtype):
        """[B, S] 0/1 mask -> [B, 1, 1, S] additive (1 - m) * -10000 (reference :798-806, Q27)."""
        return (1.0 - attention_mask[:, None, None, :].to(dtype)) * -10000.0

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, output_all_encoded_layers=True,
                checkpoint_activations=False):
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        if self._can_fuse(input_ids):
            seq2d, pooled = self.fused_forward(input_ids, token_type_ids, attention_mask, checkpoint_activations)
            seq = seq2d.view(*input_ids.shape, -1)
            return ([seq] if output_all_encoded_layers else seq), pooled
        _flush_lazy_grads(self)
        mask = self.additive_mask(attention_mask, self.embeddings.word_embeddings.weight.dtype)
        layers = self.encoder(self.embeddings(input_ids, token_type_ids), mask,
                              output_all_encoded_layers=output_all_encoded_layers,
                              checkpoint_activations=checkpoint_activations)
        pooled = self.pooler(layers[-1])
        return (layers if output_all_encoded_layers else layers[-1]), pooled

    def _amax_plan(self, extra_weights=(), extra_slots=0):
        """h3 GEMM engine: this forward's ops.gemm.AmaxPool (every GEMM weight's |max| measured now,
        one launch) and the per-layer bert_ops.LayerAmax slot maps; (None, None) on other engines.
        Slots: 0-1 the embedding output (one producer; the second stays zero), then LayerAmax.NS
        per layer, then ``extra_slots`` for the caller (the pre-training head)."""
        from hetseq_amd.ops import gemm as G

        if not G.h3_active(self.compute_dtype) or not self.embeddings.word_embeddings.weight.is_cuda:
            return None, None
        from hetseq_amd.ops.bert_ops import LayerAmax

        if not G.h3p_active(self.compute_dtype):
            store = getattr(self, "_hs_store", None)
            if store is not None:
                store.params_ready()  # (every weight's |max| is measured now, before the first layer)
        Ws = [blk._weights() for blk in self.encoder.layer]
        # (h3p engine: the layers' products need no |max| -- their slots stay reserved, unmeasured)
        weights = [None if G.h3p_active(self.compute_dtype) else w for W in Ws
                   for w in (W.wqkv, W.wo, W.w1, W.w2)] + list(extra_weights)
        L, NS = len(Ws), LayerAmax.NS
        pool = G.AmaxPool(weights, 2 + L * NS + extra_slots, self.embeddings.word_embeddings.weight.device, split=4)
        plan = []
        for i in range(L):
            la = LayerAmax()
            la.pool, la.base = pool, 2 + i * NS
            la.w = tuple(pool.w(4 * i + k) for k in range(4))
            if i == 0:  # both half-batch chains read the embedding's slot (written before the fork)
                la.x, la.xw = (pool.act(0), pool.act(0)), pool.act(0, 2)
            else:
                o = 2 + (i - 1) * NS + 6  # the previous layer's h2 halves
                la.x, la.xw = (pool.act(o), pool.act(o + 1)), pool.act(o, 2)
            plan.append(la)
        return pool, plan

    def update_groups(self):
        e = self.embeddings
        return ([list(e.parameters())] + [list(blk.parameters()) for blk in self.encoder.layer]
                + [list(self.pooler.parameters())])

    def grad_groups(self):
        """The gradient groups of the encoder layer whose backward finishes last (layer 0)."""
        return self.encoder.layer[0].grad_groups()

    def early_layer(self):
        return self.encoder.layer[0]

    def _param_ready(self, chunk):
        """Staged update (runtime/flat.py): wait for chunk ``chunk`` of the flat store -- 0 the
        embeddings, 1 + i encoder layer i, then the rest."""
        store = getattr(self, "_hs_store", None)
        if store is not None and store.chunks is not None:
            store.param_ready(chunk)

    def fused_encoder(self, input_ids, token_type_ids, attention_mask, checkpoint_activations=False, amax=None):
        """Fused embeddings + encoder: the sequence output [B*S, H] in the compute dtype.  ``amax``:
        (pool, per-layer slot maps) from :meth:`_amax_plan` (h3 engine); planned here when None."""
        from hetseq_amd.runtime.profiling import range_pop, range_push

        B, S = input_ids.shape
        mask = attention_mask.to(torch.int64).contiguous()
        pool, plan = amax if amax is not None else self._amax_plan()
        self._h3p_refresh(B * S)
        self._param_ready(0)
        range_push("embeddings")
        x = self.embeddings.fused(input_ids, token_type_ids, self.compute_dtype,
                                  amax=pool.act(0) if pool is not None else None)
        range_pop()
        from hetseq_amd.runtime import streams

        # the two half-batch chains of the split forward meet only after the last layer (the
        # tensors the second chain reads are kept alive until then: streams.chain_keep)
        with streams.fwd_chain(x.device, on=x.is_cuda):
            for i, blk in enumerate(self.encoder.layer):
                if i == 1 and pool is not None:
                    pool.wait_rest()  # layers >= 1 read weight |max| measured on the side stream
                range_push("layer%d" % i)
                self._param_ready(1 + i)  # (before the layer forks its second half-batch chain)
                x = blk.fused(x, mask, B, S, recompute=checkpoint_activations,
                              amax=plan[i] if plan is not None else None)
                range_pop()
        if pool is not None:
            pool.wait_rest()  # (one-layer models: the head's weights)
        return x

    def _h3p_refresh(self, rows):
        """h3p engine: split every layer's GEMM weights into block-scaled planes (one launch over all
        of them -- the weights change in place at every update) and hand each layer its planes; the
        layers of a forward the engine does not tile get None (they run the h3 engine)."""
        from types import SimpleNamespace

        from hetseq_amd.ops import gemm as G
        from hetseq_amd.ops import h3p

        blks = list(self.encoder.layer)
        dev = self.embeddings.word_embeddings.weight.device
        cfg = self.config
        use = (G.h3p_active(self.compute_dtype) and dev.type == "cuda" and all(b.fused_ok(None, 32) for b in blks)
               and h3p.ok_shape(rows, cfg.hidden_size, cfg.intermediate_size, 3 * cfg.hidden_size))
        if not use:
            for b in blks:
                b.__dict__["_hs_h3p_cur"] = None
            return

        cached = self.__dict__.get("_hs_h3p")
        store = getattr(self, "_hs_store", None)
        if cached is None or cached["store"] is not store or store is None:
            pairs, per, tabs = [], [], []
            for b in blks:
                b.__dict__["_hs_h3p_cur"] = None
                W = b._weights()
                hp = SimpleNamespace(**{k: h3p.empty(getattr(W, k).shape[0], getattr(W, k).shape[1], dev)
                                        for k in ("wqkv", "wo", "w1", "w2")})
                lp = [(getattr(W, k), getattr(hp, k)) for k in ("wqkv", "wo", "w1", "w2")]
                pairs += lp
                per.append(hp)
                tabs.append(h3p.SplitTable(lp, dev))
            cached = {"store": store, "all": h3p.SplitTable(pairs, dev), "per": per, "tabs": tabs,
                      "stamp": [None] * len(blks)}
            self.__dict__["_hs_h3p"] = cached
            if store is not None and store.chunks is not None:
                # every update re-splits layer i's weights right after updating them (on the updating
                # stream, before chunk 1 + i's fence: runtime/flat.py add_update_hook)
                for i in range(len(blks)):
                    store.add_update_hook(1 + i, self._h3p_hook(cached, i))
        # planes made for the current parameters are kept; the others are split now (the first
        # forward, parameters changed outside an update, no store)
        now = store.stamp() if store is not None else None
        stale = [i for i, st in enumerate(cached["stamp"]) if now is None or st != now]
        if stale:
            if store is not None:
                store.params_ready()
            if len(stale) == len(blks):
                cached["all"].run()
            else:
                for i in stale:
                    cached["tabs"][i].run()
            for i in stale:
                cached["stamp"][i] = now
        for b, hp in zip(blks, cached["per"]):
            b.__dict__["_hs_h3p_cur"] = hp

    def _h3p_hook(self, cached, i):
        store = cached["store"]

        def hook():
            from hetseq_amd.ops import gemm as G

            if self.__dict__.get("_hs_h3p") is not cached:
                return
            if G.h3p_active(self.compute_dtype):
                cached["tabs"][i].run()
                cached["stamp"][i] = store.stamp()
            else:
                cached["stamp"][i] = None  # (another engine: re-split when h3p is next used)
        return hook

    def fused_forward(self, input_ids, token_type_ids, attention_mask, checkpoint_activations=False):
        """Fused encoder + pooler: (sequence output [B*S, H], pooled [B, H])."""
        x = self.fused_encoder(input_ids, token_type_ids, attention_mask, checkpoint_activations)
        B, S = input_ids.shape
        return x, self.pooler.dense_act(x.view(B, S, -1)[:, 0])


# the masked-LM head's products on the h3p engine (BertForPreTraining._head_h3p); False: the per-tensor
# h3 engine (A/B: bench.py --ab head_h3p,head_h3)
HEAD_H3P = True
# bf16: the tied decoder's products on the plane kernels over the padded vocabulary
# (BertForPreTraining._head_bf16_pad); False: those three products on the library
HEAD_BF16_PAD = True


def _xent(logits, target, ignore_index=-100):
    """Cross-entropy in fp32 whatever the compute dtype."""
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index)


def _flush_lazy_grads(module):
    """Before a forward whose backward is not (entirely) the fused one: gradient regions a lazy
    zero_grad left pending for the fused store-mode writers (runtime/flat.py ``cover``) are cleared
    now, since autograd -- not those writers -- will accumulate into them."""
    store = getattr(module, "_hs_store", None)
    if store is not None:
        store.params_ready()  # (this forward reads parameters outside the staged-update chunks)
        store.flush_lazy()


class BertForPreTraining(BertPreTrainedModel):
    """BERT with the MLM + NSP pre-training heads; with labels, returns the summed loss."""

    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)
        self.cls = BertPreTrainingHeads(config, self.bert.embeddings.word_embeddings.weight)
        self.apply(self.init_bert_weights)
        self.max_predictions_per_seq = None  # set by the task from the data (sparse MLM capacity)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_lm_labels=None,
                next_sentence_label=None, checkpoint_activations=False):
        labelled = masked_lm_labels is not None and next_sentence_label is not None
        if labelled and self.bert._can_fuse(input_ids):
            return self._fused_loss(input_ids, token_type_ids, attention_mask, masked_lm_labels, next_sentence_label,
                                    checkpoint_activations)
        _flush_lazy_grads(self)
        seq, pooled = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False,
                                checkpoint_activations=checkpoint_activations)
        mlm_scores, nsp_scores = self.cls(seq, pooled)
        if not labelled:
            return mlm_scores, nsp_scores
        return (_xent(mlm_scores.reshape(-1, self.config.vocab_size), masked_lm_labels.reshape(-1), -1)
                + _xent(nsp_scores.reshape(-1, 2), next_sentence_label.reshape(-1), -1))

    def grad_groups(self):
        return self.bert.grad_groups()

    def early_layer(self):
        return self.bert.early_layer()

    def update_groups(self):
        """Embeddings, each encoder layer, then the pooler and heads (the tied decoder weight is the
        word embedding: chunk 0)."""
        b = self.bert
        seen = set()
        groups = []
        for ps in b.update_groups()[:-1] + [list(b.pooler.parameters()) + list(self.cls.parameters())]:
            g = [p for p in ps if id(p) not in seen]
            seen.update(id(p) for p in g)
            groups.append(g)
        return groups

    def _mlm_weights(self):
        t = self.cls.predictions.transform
        wt, wd = t.dense_act.weight, self.cls.predictions.decoder.weight
        store = getattr(self, "_hs_store", None)
        if self.compute_dtype != torch.bfloat16:
            return wt.detach(), wd.detach()
        if store is not None:
            return store.shadow_view(wt), store.shadow_view(wd)
        return wt.detach().bfloat16(), wd.detach().bfloat16()

    def _head_h3p(self):
        """h3p engine: the masked-LM head's GEMM weights as block-scaled planes -- the transform's
        [H, H] and the tied decoder's [V, H] padded to pad512(V) rows (the missing rows split as zeros)
        -- or None (another engine, a CPU model, widths the engine does not tile).  Re-split right after
        every update of their chunks (the word table is chunk 0, the transform the heads' last chunk:
        runtime/flat.py add_update_hook, on the updating stream), else here when stale."""
        from hetseq_amd.ops import gemm as G
        from hetseq_amd.ops import h3p

        wt = self.cls.predictions.transform.dense_act.weight
        wd = self.cls.predictions.decoder.weight
        H, V = wt.shape[0], wd.shape[0]
        if not (HEAD_H3P and G.h3p_active(self.compute_dtype) and wt.is_cuda and H % 128 == 0
                and wt.dtype == torch.float32):
            return None
        store = getattr(self, "_hs_store", None)
        cached = self.__dict__.get("_hs_head_h3p")
        if cached is None or cached["store"] is not store:
            Vp = (V + 511) // 512 * 512
            tp, dp = h3p.empty(H, H, wt.device), h3p.empty(Vp, H, wt.device)
            tabs = [h3p.SplitTable([(wd.detach(), dp)], wt.device), h3p.SplitTable([(wt.detach(), tp)], wt.device)]
            cached = {"store": store, "planes": (tp, dp), "tabs": tabs, "stamp": [None, None]}
            self.__dict__["_hs_head_h3p"] = cached
            if store is not None and store.chunks is not None:
                from hetseq_amd.runtime.flat import bisect_chunk

                for k, w in enumerate((wd, wt)):
                    store.add_update_hook(bisect_chunk(store.chunks, store.offset(w)), self._head_h3p_hook(cached, k))
        now = store.stamp() if store is not None else None
        for k in range(2):
            if now is None or cached["stamp"][k] != now:
                if store is not None:
                    store.params_ready()
                cached["tabs"][k].run()
                cached["stamp"][k] = now
        return cached["planes"]

    def _head_bf16_pad(self):
        """bf16 engine: the tied decoder's bf16 weight copied into a [pad512(V), H] buffer whose rows past
        V are zero, plus an fp32 bias buffer of pad512(V) (zero past V): the hand-written plane kernels
        tile only multiples of 128, so the vocabulary products run padded instead of on the library.
        The copy is refreshed right after every update of the word table's chunk (its update hook, on
        the updating stream), else here when stale.  None: another engine or a CPU model."""
        from hetseq_amd.ops import gemm as G

        wd = self.cls.predictions.decoder.weight
        V, H = wd.shape
        if not (HEAD_BF16_PAD and self.compute_dtype == torch.bfloat16 and wd.is_cuda and H % 128 == 0
                and G.gemm_mode() != "blas"):
            return None
        store = getattr(self, "_hs_store", None)
        cached = self.__dict__.get("_hs_head_bf16")
        if cached is None or cached["store"] is not store:
            Vp = (V + 511) // 512 * 512
            cached = {"store": store, "w": torch.zeros((Vp, H), dtype=torch.bfloat16, device=wd.device),
                      "b": torch.zeros(Vp, dtype=torch.float32, device=wd.device), "stamp": None}
            self.__dict__["_hs_head_bf16"] = cached
            if store is not None and store.chunks is not None:
                from hetseq_amd.runtime.flat import bisect_chunk

                store.add_update_hook(bisect_chunk(store.chunks, store.offset(wd)), self._head_bf16_hook(cached))
        now = store.stamp() if store is not None else None
        if now is None or cached["stamp"] != now:
            if store is not None:
                store.params_ready()
            cached["w"][:V].copy_(self._mlm_weights()[1])
            cached["stamp"] = now
        return cached["w"], cached["b"]

    def _head_bf16_hook(self, cached):
        store = cached["store"]

        def hook():
            if self.__dict__.get("_hs_head_bf16") is not cached or self.compute_dtype != torch.bfloat16:
                return
            wd = self.cls.predictions.decoder.weight
            cached["w"][:wd.shape[0]].copy_(store.shadow_view(wd))
            cached["stamp"] = store.stamp()
        return hook

    def _head_h3p_hook(self, cached, k):
        store = cached["store"]

        def hook():
            from hetseq_amd.ops import gemm as G

            if self.__dict__.get("_hs_head_h3p") is not cached:
                return
            if G.h3p_active(self.compute_dtype):
                cached["tabs"][k].run()
                cached["stamp"][k] = store.stamp()
            else:
                cached["stamp"][k] = None
        return hook

    def sparse_embedding(self):
        """(tables, rest) for the data-parallel engine's sparse table exchange (parallel/tied.py):
        the word / position / token-type tables, whose gradient rows the fused embedding backward
        hands over (the word table also takes the tied decoder's dense gradient, signalled by the
        fused loss), and the rest of the embedding module (its LayerNorm)."""
        e = self.bert.embeddings
        return ([e.word_embeddings.weight, e.position_embeddings.weight, e.token_type_embeddings.weight],
                [e.LayerNorm.weight, e.LayerNorm.bias])

    def _fused_loss(self, input_ids, token_type_ids, attention_mask, labels, nsp_label, checkpoint_activations):
        from hetseq_amd.ops.bert_ops import FusedPreTrainingLoss

        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        B, S = input_ids.shape
        wt_, wd_ = self._mlm_weights()
        head_hp = self._head_h3p()
        head_bf = self._head_bf16_pad() if head_hp is None else None
        head_w = (wt_, wd_) if isinstance(wt_, torch.Tensor) and wt_.dtype == torch.float32 and head_hp is None else ()
        pool, plan = self.bert._amax_plan(extra_weights=head_w, extra_slots=3)
        seq2d = self.bert.fused_encoder(input_ids, token_type_ids, attention_mask, checkpoint_activations,
                                        amax=(pool, plan))
        cap = B * S if self.max_predictions_per_seq is None else min(B * S, B * int(self.max_predictions_per_seq))
        if head_hp is not None or head_bf is not None:
            cap = (cap + 127) // 128 * 128  # (rows past the labelled ones: zero rows, label -1, no loss / gradient)
        t, pred = self.cls.predictions.transform, self.cls.predictions
        pooler, nsp = self.bert.pooler.dense_act, self.cls.seq_relationship
        params = [t.dense_act.weight, t.dense_act.bias, t.LayerNorm.weight, t.LayerNorm.bias, pred.decoder.weight,
                  pred.bias, pooler.weight, pooler.bias, nsp.weight, nsp.bias]
        meta = {"cap": cap, "eps": t.LayerNorm.variance_epsilon, "weights": self._mlm_weights, "B": B, "S": S}
        if head_hp is not None:
            meta["h3p"] = head_hp
        if head_bf is not None:
            meta["bf16pad"] = head_bf
        if pool is not None and head_w:
            L = len(plan)
            last = plan[-1]
            # h3 slots of the head: the sequence output (last layer's h2 halves), the transform and
            # decoder weights, and the transform LN output t2 (the decoder's A operand)
            meta["amax"] = {"seq": last.a(6, 2), "wt": pool.w(4 * L), "wd": pool.w(4 * L + 1),
                            "t2": pool.act(2 + L * last.NS), "dl": pool.act(2 + L * last.NS + 1),
                            "dt": pool.act(2 + L * last.NS + 2)}
        store = getattr(self, "_hs_store", None)
        if store is not None:
            meta["grad_sink"] = lambda: [store.grad_view(q) for q in params]
            meta["store"] = store
            store.cover(store.grad_view(pred.decoder.weight))  # the tied decoder's gradient store (lazy zero_grad)
            if store.chunks is not None:
                store.param_ready(len(store.chunks) - 1)  # the heads' chunk (and the deferred zero_grad)
        if pool is not None:
            pool.measure_deferred()  # (h3p engine: the head weights' |max|, now that they are current)
        return FusedPreTrainingLoss.apply(seq2d, labels.reshape(-1).contiguous(), nsp_label.reshape(-1).contiguous(),
                                          meta, *params)


# ----------------------------------------------------------------- fine-tuning heads (reference :891-1301)
class _BertFineTune(BertPreTrainedModel):
    """An encoder plus a task head; subclasses define the head modules and ``_head``."""

    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)

    def _encode(self, input_ids, token_type_ids, attention_mask):
        return self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)


class BertForMaskedLM(_BertFineTune):
    def __init__(self, config):
        super().__init__(config)
        self.cls = BertOnlyMLMHead(config, self.bert.embeddings.word_embeddings.weight)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_lm_labels=None,
                checkpoint_activations=False):
        scores = self.cls(self._encode(input_ids, token_type_ids, attention_mask)[0])
        if masked_lm_labels is None:
            return scores
        return _xent(scores.reshape(-1, self.config.vocab_size), masked_lm_labels.reshape(-1), -1)


class BertForNextSentencePrediction(_BertFineTune):
    def __init__(self, config):
        super().__init__(config)
        self.cls = BertOnlyNSPHead(config)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, next_sentence_label=None,
                checkpoint_activations=False):
        scores = self.cls(self._encode(input_ids, token_type_ids, attention_mask)[1])
        if next_sentence_label is None:
            return scores
        return _xent(scores.reshape(-1, 2), next_sentence_label.reshape(-1), -1)


class _PooledClassifier(_BertFineTune):
    """dropout(pooled) -> Linear(H, width)."""

    def __init__(self, config, width):
        super().__init__(config)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.classifier = nn.Linear(config.hidden_size, width)
        self.apply(self.init_bert_weights)

    def _logits(self, input_ids, token_type_ids, attention_mask):
        return self.classifier(self.dropout(self._encode(input_ids, token_type_ids, attention_mask)[1]))


class BertForSequenceClassification(_PooledClassifier):
    def __init__(self, config, num_labels):
        super().__init__(config, num_labels)
        self.num_labels = num_labels

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None, checkpoint_activations=False):
        logits = self._logits(input_ids, token_type_ids, attention_mask)
        return logits if labels is None else _xent(logits.reshape(-1, self.num_labels), labels.reshape(-1))


class BertForMultipleChoice(_PooledClassifier):
    """Scores each of ``num_choices`` [B, C, S] candidates with a 1-wide classifier."""

    def __init__(self, config, num_choices):
        super().__init__(config, 1)
        self.num_choices = num_choices

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None, checkpoint_activations=False):
        S = input_ids.shape[-1]
        flat = [t.reshape(-1, S) if t is not None else None for t in (input_ids, token_type_ids, attention_mask)]
        logits = self._logits(*flat).reshape(-1, self.num_choices)
        return logits if labels is None else _xent(logits, labels)


class BertForTokenClassification(_BertFineTune):
    def __init__(self, config, num_labels):
        super().__init__(config)
        self.num_labels = num_labels
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.classifier = nn.Linear(config.hidden_size, num_labels)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None, checkpoint_activations=False):
        seq = self._encode(input_ids, token_type_ids, attention_mask)[0]
        logits = self.classifier(self.dropout(seq)).reshape(-1, self.num_labels)
        if labels is None:
            return logits.view(*seq.shape[:-1], self.num_labels)
        labels = labels.reshape(-1)
        if attention_mask is not None:  # only positions the mask keeps
            keep = attention_mask.reshape(-1) == 1
            logits, labels = logits[keep], labels[keep]
        return _xent(logits, labels)


class BertForQuestionAnswering(_BertFineTune):
    """Span start / end logits; positions outside the sequence are clamped to S and ignored."""

    def __init__(self, config):
        super().__init__(config)
        self.qa_outputs = nn.Linear(config.hidden_size, 2)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, start_positions=None, end_positions=None,
                checkpoint_activations=False):
        seq = self._encode(input_ids, token_type_ids, attention_mask)[0]
        start_logits, end_logits = self.qa_outputs(seq).unbind(-1)
        if start_positions is None or end_positions is None:
            return start_logits, end_logits
        S = start_logits.shape[1]
        losses = [_xent(lg, pos.reshape(pos.shape[0], -1)[:, 0].clamp(0, S), ignore_index=S)
                  for lg, pos in ((start_logits, start_positions), (end_logits, end_positions))]
        return sum(losses) / 2
