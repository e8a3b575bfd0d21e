"""BERT model family.

Module tree, parameter names (207 state-dict keys for BERT-base, tied MLM
decoder), initialisation and forward semantics follow the reference
(reference: bert_modeling.py:180-1301):
  * post-LN encoder, separate Q/K/V Linear layers, additive (1-mask)*-10000
    attention mask (Q27), dropout on attention probabilities;
  * erf-GELU with the 1.41421 constant (Q18); TF-style LayerNorm, eps 1e-12;
  * ``LinearActivation`` keeps kaiming-uniform init with non-zero bias and is
    deep-copied across layers (Q17); ``init_bert_weights`` N(0, 0.02) for
    Linear/Embedding, applied by BertModel and again by the heads model;
  * ``BertForPreTraining(...)`` returns MLM CE(ignore -1) + NSP CE.
  * fine-tuning heads: MaskedLM, NextSentencePrediction, SequenceClassification,
    MultipleChoice, TokenClassification, QuestionAnswering.

Two execution paths share these modules:
  * fused (GPU): ``FusedEmbedding`` -> 12 x ``FusedBertLayer`` -> ``FusedMLMLoss``
    over the gfx950 HIP kernels (hetseq_amd/ops/bert_ops.py), fp32 or bf16
    compute (``attach_store``/``set_compute_dtype``);
  * reference (CPU or ``--no-fused``): plain torch ops, mathematically the
    reference model; also the numerical oracle for the kernel tests.
"""
from __future__ import annotations

import copy
import json
import logging
import math
import os
import tarfile
import tempfile

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn import CrossEntropyLoss
from torch.nn import init
from torch.nn.parameter import Parameter
from torch.utils import checkpoint

logger = logging.getLogger(__name__)

TF_WEIGHTS_NAME = "model.ckpt"
CONFIG_NAME = "bert_config.json"
WEIGHTS_NAME = "pytorch_model.bin"


# ----------------------------------------------------------------- activations
def f_gelu(x):
    return x * 0.5 * (1.0 + torch.erf(x / 1.41421))


def bias_gelu(bias, y):
    x = bias + y
    return x * 0.5 * (1.0 + torch.erf(x / 1.41421))


def bias_tanh(bias, y):
    return torch.tanh(bias + y)


def gelu(x):
    return f_gelu(x)


def swish(x):
    return x * torch.sigmoid(x)


ACT2FN = {"gelu": gelu, "relu": torch.nn.functional.relu, "swish": swish}


def _fused_ok(t):
    from hetseq_amd.ops._C import use_fused

    return use_fused(t)


class LinearActivation(nn.Module):
    """Linear (bias-free GEMM) followed by a fused bias+activation."""

    __constants__ = ["bias"]

    def __init__(self, in_features, out_features, act="gelu", bias=True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.fused_gelu = False
        self.fused_tanh = False
        self.act = act
        if isinstance(act, str):
            if bias and act == "gelu":
                self.fused_gelu = True
            elif bias and act == "tanh":
                self.fused_tanh = True
            else:
                self.act_fn = ACT2FN[act]
        else:
            self.act_fn = act
        self.weight = Parameter(torch.empty(out_features, in_features))
        if bias:
            self.bias = Parameter(torch.empty(out_features))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in, _ = init._calculate_fan_in_and_fan_out(self.weight)
            bound = 1 / math.sqrt(fan_in)
            init.uniform_(self.bias, -bound, bound)

    def forward(self, input):
        if self.fused_gelu:
            if _fused_ok(input) and input.dim() == 2 and self.out_features % 4 == 0:
                from hetseq_amd.ops.bert_ops import bias_gelu as fused_bias_gelu

                return fused_bias_gelu(F.linear(input, _cw(self.weight, input)), self.bias)
            return bias_gelu(self.bias, F.linear(input, _cw(self.weight, input), None))
        elif self.fused_tanh:
            return bias_tanh(self.bias, F.linear(input, _cw(self.weight, input), None))
        return self.act_fn(F.linear(input, _cw(self.weight, input), self.bias))

    def extra_repr(self):
        return "in_features={}, out_features={}, bias={}".format(self.in_features, self.out_features,
                                                                  self.bias is not None)


def _cw(w, x):
    """Weight in the compute dtype of ``x`` (autograd-transparent cast)."""
    return w if w.dtype == x.dtype else w.to(x.dtype)


# ----------------------------------------------------------------- config
class BertConfig(object):
    """Configuration of a BertModel (same JSON keys as the reference)."""

    def __init__(self, vocab_size_or_config_json_file, hidden_size=768, num_hidden_layers=12,
                 num_attention_heads=12, intermediate_size=3072, hidden_act="gelu", hidden_dropout_prob=0.1,
                 attention_probs_dropout_prob=0.1, max_position_embeddings=512, type_vocab_size=2,
                 initializer_range=0.02):
        if isinstance(vocab_size_or_config_json_file, str):
            with open(vocab_size_or_config_json_file, "r", encoding="utf-8") as reader:
                json_config = json.loads(reader.read())
            for key, value in json_config.items():
                self.__dict__[key] = value
        elif isinstance(vocab_size_or_config_json_file, int):
            self.vocab_size = vocab_size_or_config_json_file
            self.hidden_size = hidden_size
            self.num_hidden_layers = num_hidden_layers
            self.num_attention_heads = num_attention_heads
            self.hidden_act = hidden_act
            self.intermediate_size = intermediate_size
            self.hidden_dropout_prob = hidden_dropout_prob
            self.attention_probs_dropout_prob = attention_probs_dropout_prob
            self.max_position_embeddings = max_position_embeddings
            self.type_vocab_size = type_vocab_size
            self.initializer_range = initializer_range
        else:
            raise ValueError("First argument must be either a vocabulary size (int) or the path to a pretrained "
                             "model config file (str)")

    @classmethod
    def from_dict(cls, json_object):
        config = BertConfig(vocab_size_or_config_json_file=-1)
        for key, value in json_object.items():
            config.__dict__[key] = value
        return config

    @classmethod
    def from_json_file(cls, json_file):
        with open(json_file, "r", encoding="utf-8") as reader:
            text = reader.read()
        return cls.from_dict(json.loads(text))

    def __repr__(self):
        return str(self.to_json_string())

    def to_dict(self):
        return copy.deepcopy(self.__dict__)

    def to_json_string(self):
        return json.dumps(self.to_dict(), indent=2, sort_keys=True) + "\n"


class BertLayerNorm(nn.Module):
    """TF-style LayerNorm (epsilon inside the square root), eps=1e-12."""

    def __init__(self, hidden_size, eps=1e-12):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size))
        self.bias = nn.Parameter(torch.zeros(hidden_size))
        self.variance_epsilon = eps

    def forward(self, x):
        if _fused_ok(x) and x.shape[-1] in (256, 512, 768, 1024, 1536, 2048):
            from hetseq_amd.ops.bert_ops import layer_norm

            shp = x.shape
            return layer_norm(x.reshape(-1, shp[-1]).contiguous(), self.weight, self.bias,
                              self.variance_epsilon).view(shp)
        u = x.mean(-1, keepdim=True)
        s = (x - u).pow(2).mean(-1, keepdim=True)
        x = (x - u) / torch.sqrt(s + self.variance_epsilon)
        return self.weight * x + self.bias


# ----------------------------------------------------------------- modules
class BertEmbeddings(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.word_embeddings = nn.Embedding(config.vocab_size, config.hidden_size)
        self.position_embeddings = nn.Embedding(config.max_position_embeddings, config.hidden_size)
        self.token_type_embeddings = nn.Embedding(config.type_vocab_size, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=1e-12)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, input_ids, token_type_ids=None):
        seq_length = input_ids.size(1)
        position_ids = torch.arange(seq_length, dtype=torch.long, device=input_ids.device)
        position_ids = position_ids.unsqueeze(0).expand_as(input_ids)
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        embeddings = (self.word_embeddings(input_ids) + self.position_embeddings(position_ids)
                      + self.token_type_embeddings(token_type_ids))
        embeddings = self.LayerNorm(embeddings)
        return self.dropout(embeddings)

    def fused(self, input_ids, token_type_ids, out_dtype):
        from hetseq_amd.ops.bert_ops import FusedEmbedding

        p = self.dropout.p if self.training else 0.0
        params = [self.word_embeddings.weight, self.position_embeddings.weight, self.token_type_embeddings.weight,
                  self.LayerNorm.weight, self.LayerNorm.bias]
        store = getattr(self, "_hs_store", None)
        sink = None
        if store is not None:
            sink = {"views": lambda: [store.grad_view(q) for q in params]}
        return FusedEmbedding.apply(input_ids, token_type_ids, *params, p, self.LayerNorm.variance_epsilon,
                                    out_dtype, sink)


class BertSelfAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        if config.hidden_size % config.num_attention_heads != 0:
            raise ValueError("The hidden size (%d) is not a multiple of the number of attention heads (%d)"
                             % (config.hidden_size, config.num_attention_heads))
        self.num_attention_heads = config.num_attention_heads
        self.attention_head_size = int(config.hidden_size / config.num_attention_heads)
        self.all_head_size = self.num_attention_heads * self.attention_head_size
        self.query = nn.Linear(config.hidden_size, self.all_head_size)
        self.key = nn.Linear(config.hidden_size, self.all_head_size)
        self.value = nn.Linear(config.hidden_size, self.all_head_size)
        self.dropout = nn.Dropout(config.attention_probs_dropout_prob)
        self.softmax = nn.Softmax(dim=-1)
        # Q/K/V weights (and biases) adjacent in the flat store -> one [3H, H] GEMM operand
        self._flat_groups = [[self.query.weight, self.key.weight, self.value.weight],
                             [self.query.bias, self.key.bias, self.value.bias]]

    def transpose_for_scores(self, x):
        new_x_shape = x.size()[:-1] + (self.num_attention_heads, self.attention_head_size)
        return x.view(*new_x_shape).permute(0, 2, 1, 3)

    def transpose_key_for_scores(self, x):
        new_x_shape = x.size()[:-1] + (self.num_attention_heads, self.attention_head_size)
        return x.view(*new_x_shape).permute(0, 2, 3, 1)

    def forward(self, hidden_states, attention_mask):
        q = self.transpose_for_scores(self.query(hidden_states))
        k = self.transpose_key_for_scores(self.key(hidden_states))
        v = self.transpose_for_scores(self.value(hidden_states))
        scores = torch.matmul(q, k) / math.sqrt(self.attention_head_size)
        scores = scores + attention_mask
        probs = self.dropout(self.softmax(scores))
        ctx = torch.matmul(probs, v).permute(0, 2, 1, 3).contiguous()
        return ctx.view(*(ctx.size()[:-2] + (self.all_head_size,)))


class BertSelfOutput(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=1e-12)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, hidden_states, input_tensor):
        hidden_states = self.dropout(self.dense(hidden_states))
        return self.LayerNorm(hidden_states + input_tensor)


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


class BertOutput(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.intermediate_size, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=1e-12)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, hidden_states, input_tensor):
        hidden_states = self.dropout(self.dense(hidden_states))
        return self.LayerNorm(hidden_states + input_tensor)


class BertLayer(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.attention = BertAttention(config)
        self.intermediate = BertIntermediate(config)
        self.output = BertOutput(config)

    def forward(self, hidden_states, attention_mask):
        attention_output = self.attention(hidden_states, attention_mask)
        intermediate_output = self.intermediate(attention_output)
        return self.output(intermediate_output, attention_output)

    # ------------------------------------------------------------- fused path
    def fused_params(self):
        cached = self.__dict__.get("_hs_pcache")  # parameter objects never change identity
        if cached is not None:
            return cached
        a, o = self.attention, self.output
        self.__dict__["_hs_pcache"] = ps = [a.self.query.weight, a.self.query.bias, a.self.key.weight, a.self.key.bias, a.self.value.weight,
                a.self.value.bias, a.output.dense.weight, a.output.dense.bias, a.output.LayerNorm.weight,
                a.output.LayerNorm.bias, self.intermediate.dense_act.weight, self.intermediate.dense_act.bias,
                o.dense.weight, o.dense.bias, o.LayerNorm.weight, o.LayerNorm.bias]
        return ps

    def _weights(self):
        """Kernel-side weight views.  With a flat store they are fixed views into its buffers
        (parameters are updated in place), so they are built once and cached."""
        cached = getattr(self, "_hs_wcache", None)
        if cached is not None:
            return cached
        W = self._build_weights()
        if getattr(self, "_hs_store", None) is not None:
            self._hs_wcache = W
        return W

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

    def fused_ok(self, x, S):
        sa = self.attention.self
        H = sa.query.weight.shape[1]
        return (sa.attention_head_size == 64 and H in (256, 512, 768, 1024, 1536, 2048) and S % 32 == 0
                and self.intermediate.dense_act.fused_gelu and self.intermediate.dense_act.out_features % 4 == 0)

    def fused(self, x2d, mask_i64, B, S, recompute=False):
        from hetseq_amd.ops.bert_ops import FusedBertLayer
        from hetseq_amd.runtime import rng

        p_h = self.output.dropout.p if self.training else 0.0
        p_a = self.attention.self.dropout.p if self.training else 0.0
        seeds = tuple(rng.fork() if p > 0 else (0, 0) for p in (p_a, p_h, p_h))
        cfg = (B, S, self.attention.self.num_attention_heads, p_h, p_a, self.output.LayerNorm.variance_epsilon, seeds)
        meta = {"weights": self._weights, "cfg": cfg, "recompute": recompute}
        store = getattr(self, "_hs_store", None)
        if store is not None:
            meta["grad_sink"] = self._grad_views
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
        return g


class BertEncoder(nn.Module):
    def __init__(self, config):
        super().__init__()
        layer = BertLayer(config)
        self.layer = nn.ModuleList([copy.deepcopy(layer) for _ in range(config.num_hidden_layers)])

    def forward(self, hidden_states, attention_mask, output_all_encoded_layers=True, checkpoint_activations=False):
        all_encoder_layers = []

        def custom(start, end):
            def custom_forward(*inputs):
                x_ = inputs[0]
                for layer in self.layer[start:end]:
                    x_ = layer(x_, inputs[1])
                return x_

            return custom_forward

        if checkpoint_activations:
            l, num_layers = 0, len(self.layer)
            chunk_length = math.ceil(math.sqrt(num_layers))
            while l < num_layers:
                hidden_states = checkpoint.checkpoint(custom(l, l + chunk_length), hidden_states, attention_mask * 1,
                                                      use_reentrant=False)
                l += chunk_length
        else:
            for layer_module in self.layer:
                hidden_states = layer_module(hidden_states, attention_mask)
                if output_all_encoded_layers:
                    all_encoder_layers.append(hidden_states)
        if not output_all_encoded_layers or checkpoint_activations:
            all_encoder_layers.append(hidden_states)
        return all_encoder_layers


class BertPooler(nn.Module):
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
    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        self.transform = BertPredictionHeadTransform(config)
        self.decoder = nn.Linear(bert_model_embedding_weights.size(1), bert_model_embedding_weights.size(0),
                                 bias=False)
        self.decoder.weight = bert_model_embedding_weights
        self.bias = nn.Parameter(torch.zeros(bert_model_embedding_weights.size(0)))

    def forward(self, hidden_states):
        hidden_states = self.transform(hidden_states)
        from hetseq_amd.runtime.profiling import range_push, range_pop

        range_push("decoder")
        out = self.decoder(hidden_states) + self.bias
        range_pop()
        return out


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
    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        self.predictions = BertLMPredictionHead(config, bert_model_embedding_weights)
        self.seq_relationship = nn.Linear(config.hidden_size, 2)

    def forward(self, sequence_output, pooled_output):
        return self.predictions(sequence_output), self.seq_relationship(pooled_output)


class BertPreTrainedModel(nn.Module):
    """Weight init + (local-only) ``from_pretrained``."""

    def __init__(self, config, *inputs, **kwargs):
        super().__init__()
        if not isinstance(config, BertConfig):
            raise ValueError("Parameter config in `{}(config)` should be an instance of class `BertConfig`."
                             .format(self.__class__.__name__))
        self.config = config

    def init_bert_weights(self, module):
        if isinstance(module, (nn.Linear, nn.Embedding)):
            module.weight.data.normal_(mean=0.0, std=self.config.initializer_range)
        elif isinstance(module, BertLayerNorm):
            module.bias.data.zero_()
            module.weight.data.fill_(1.0)
        if isinstance(module, nn.Linear) and module.bias is not None:
            module.bias.data.zero_()

    # --- runtime plumbing (flat store / compute dtype / fused switch)
    def attach_store(self, store, compute_dtype=torch.float32):
        for m in self.modules():
            m._hs_store = store
            m._hs_dtype = compute_dtype
            m._hs_wcache = None
        self._compute_dtype = compute_dtype

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
        """Load from a local directory or .tar.gz archive holding bert_config.json + pytorch_model.bin.

        There is no network here: remote names go through
        :func:`hetseq_amd.utils.file_utils.cached_path`, which only resolves
        cached or local files.  Weights load with ``weights_only=True``."""
        from hetseq_amd.utils.file_utils import cached_path

        resolved = cached_path(pretrained_model_name_or_path, cache_dir=cache_dir)
        tempdir = None
        if os.path.isdir(resolved) or from_tf:
            serialization_dir = resolved
        else:
            tempdir = tempfile.mkdtemp()
            with tarfile.open(resolved, "r:gz") as archive:
                archive.extractall(tempdir, filter="data")
            serialization_dir = tempdir
        config = BertConfig.from_json_file(os.path.join(serialization_dir, CONFIG_NAME))
        model = cls(config, *inputs, **kwargs)
        if state_dict is None and not from_tf:
            state_dict = torch.load(os.path.join(serialization_dir, WEIGHTS_NAME), map_location="cpu",
                                    weights_only=True)
        if tempdir:
            import shutil

            shutil.rmtree(tempdir, ignore_errors=True)
        if from_tf:
            # reference: bert_modeling.py:685-688 (TF_WEIGHTS_NAME = 'model.ckpt'); read without TensorFlow
            from hetseq_amd.utils.tf_checkpoint import load_tf_weights_in_bert

            prefix = os.path.join(serialization_dir, TF_WEIGHTS_NAME)
            if not os.path.exists(prefix + ".index") and os.path.exists(os.path.join(serialization_dir,
                                                                                    "bert_model.ckpt.index")):
                prefix = os.path.join(serialization_dir, "bert_model.ckpt")  # Google's release name
            return load_tf_weights_in_bert(model, prefix)
        renamed = {}
        for k, v in state_dict.items():
            nk = k.replace("gamma", "weight").replace("beta", "bias")
            renamed[nk] = v
        missing, unexpected, errors = [], [], []
        metadata = getattr(state_dict, "_metadata", None)
        state_dict = renamed
        if metadata is not None:
            state_dict._metadata = metadata

        def load(module, prefix=""):
            local_metadata = {} if metadata is None else metadata.get(prefix[:-1], {})
            module._load_from_state_dict(state_dict, prefix, local_metadata, True, missing, unexpected, errors)
            for name, child in module._modules.items():
                if child is not None:
                    load(child, prefix + name + ".")

        start_prefix = ""
        if not hasattr(model, "bert") and any(s.startswith("bert.") for s in state_dict.keys()):
            start_prefix = "bert."
        load(model, prefix=start_prefix)
        if missing:
            logger.info("Weights of %s not initialized from pretrained model: %s", model.__class__.__name__, missing)
        if unexpected:
            logger.info("Weights from pretrained model not used in %s: %s", model.__class__.__name__, unexpected)
        if errors:
            raise RuntimeError("Error(s) in loading state_dict for {}:\n\t{}".format(model.__class__.__name__,
                                                                                      "\n\t".join(errors)))
        return model


class BertModel(BertPreTrainedModel):
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
        H = self.config.hidden_size
        return (H in (256, 512, 768, 1024, 1536, 2048) and all(l.fused_ok(None, S) for l in self.encoder.layer))

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, output_all_encoded_layers=True,
                checkpoint_activations=False):
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        if self._can_fuse(input_ids):
            seq2d, pooled = self.fused_forward(input_ids, token_type_ids, attention_mask, checkpoint_activations)
            B, S = input_ids.shape
            seq = seq2d.view(B, S, -1)
            return (seq if not output_all_encoded_layers else [seq]), pooled
        extended = attention_mask.unsqueeze(1).unsqueeze(2)
        extended = extended.to(dtype=next(self.parameters()).dtype)
        extended = (1.0 - extended) * -10000.0
        embedding_output = self.embeddings(input_ids, token_type_ids)
        encoded_layers = self.encoder(embedding_output, extended, output_all_encoded_layers=output_all_encoded_layers,
                                      checkpoint_activations=checkpoint_activations)
        sequence_output = encoded_layers[-1]
        pooled_output = self.pooler(sequence_output)
        if not output_all_encoded_layers:
            encoded_layers = encoded_layers[-1]
        return encoded_layers, pooled_output

    def fused_forward(self, input_ids, token_type_ids, attention_mask, checkpoint_activations=False):
        """Fused encoder: returns (sequence_output [B*S, H], pooled [B, H])."""
        from hetseq_amd.runtime.profiling import range_pop, range_push

        B, S = input_ids.shape
        mask = attention_mask.to(torch.int64).contiguous()
        range_push("embeddings")
        x = self.embeddings.fused(input_ids, token_type_ids, self.compute_dtype)
        range_pop()
        for i, layer in enumerate(self.encoder.layer):
            range_push("layer%d" % i)
            x = layer.fused(x, mask, B, S, recompute=checkpoint_activations)
            range_pop()
        first = x.view(B, S, -1)[:, 0]
        pooled = self.pooler.dense_act(first)
        return x, pooled


class BertForPreTraining(BertPreTrainedModel):
    """BERT with the MLM + NSP pre-training heads; returns the summed loss."""

    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)
        self.cls = BertPreTrainingHeads(config, self.bert.embeddings.word_embeddings.weight)
        self.apply(self.init_bert_weights)
        self.max_predictions_per_seq = None  # set by the task from the data (sparse MLM capacity)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_lm_labels=None,
                next_sentence_label=None, checkpoint_activations=False):
        if (masked_lm_labels is not None and next_sentence_label is not None
                and self.bert._can_fuse(input_ids)):
            return self._fused_loss(input_ids, token_type_ids, attention_mask, masked_lm_labels, next_sentence_label,
                                    checkpoint_activations)
        sequence_output, pooled_output = self.bert(input_ids, token_type_ids, attention_mask,
                                                   output_all_encoded_layers=False,
                                                   checkpoint_activations=checkpoint_activations)
        prediction_scores, seq_relationship_score = self.cls(sequence_output, pooled_output)
        if masked_lm_labels is not None and next_sentence_label is not None:
            loss_fct = CrossEntropyLoss(ignore_index=-1)
            masked_lm_loss = loss_fct(prediction_scores.view(-1, self.config.vocab_size).float(),
                                      masked_lm_labels.view(-1))
            next_sentence_loss = loss_fct(seq_relationship_score.view(-1, 2).float(), next_sentence_label.view(-1))
            return masked_lm_loss + next_sentence_loss
        return prediction_scores, seq_relationship_score

    def _mlm_weights(self):
        t = self.cls.predictions.transform
        store = getattr(self, "_hs_store", None)
        if self.compute_dtype == torch.bfloat16:
            if store is not None:
                return store.shadow_view(t.dense_act.weight), store.shadow_view(self.cls.predictions.decoder.weight)
            return t.dense_act.weight.detach().bfloat16(), self.cls.predictions.decoder.weight.detach().bfloat16()
        return t.dense_act.weight.detach(), self.cls.predictions.decoder.weight.detach()

    def _fused_loss(self, input_ids, token_type_ids, attention_mask, labels, nsp_label, checkpoint_activations):
        from hetseq_amd.ops.bert_ops import FusedMLMLoss

        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        B, S = input_ids.shape
        seq2d, pooled = self.bert.fused_forward(input_ids, token_type_ids, attention_mask, checkpoint_activations)
        cap = B * S if self.max_predictions_per_seq is None else min(B * S, B * int(self.max_predictions_per_seq))
        t = self.cls.predictions.transform
        meta = {"cap": cap, "eps": t.LayerNorm.variance_epsilon, "weights": self._mlm_weights}
        store = getattr(self, "_hs_store", None)
        if store is not None:
            cls_params = [t.dense_act.weight, t.dense_act.bias, t.LayerNorm.weight, t.LayerNorm.bias,
                          self.cls.predictions.decoder.weight, self.cls.predictions.bias]
            meta["grad_sink"] = lambda: [store.grad_view(q) for q in cls_params]
        mlm_loss = FusedMLMLoss.apply(seq2d, labels.reshape(-1).contiguous(), meta, t.dense_act.weight,
                                      t.dense_act.bias, t.LayerNorm.weight, t.LayerNorm.bias,
                                      self.cls.predictions.decoder.weight, self.cls.predictions.bias)
        nsp_logits = self.cls.seq_relationship(pooled.float() if pooled.dtype != torch.float32 else pooled)
        nsp_loss = F.cross_entropy(nsp_logits.view(-1, 2), nsp_label.view(-1), ignore_index=-1)
        return mlm_loss + nsp_loss


class BertForMaskedLM(BertPreTrainedModel):
    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)
        self.cls = BertOnlyMLMHead(config, self.bert.embeddings.word_embeddings.weight)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_lm_labels=None,
                checkpoint_activations=False):
        sequence_output, _ = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)
        prediction_scores = self.cls(sequence_output)
        if masked_lm_labels is not None:
            return CrossEntropyLoss(ignore_index=-1)(prediction_scores.view(-1, self.config.vocab_size).float(),
                                                     masked_lm_labels.view(-1))
        return prediction_scores


class BertForNextSentencePrediction(BertPreTrainedModel):
    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)
        self.cls = BertOnlyNSPHead(config)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, next_sentence_label=None,
                checkpoint_activations=False):
        _, pooled_output = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)
        seq_relationship_score = self.cls(pooled_output)
        if next_sentence_label is not None:
            return CrossEntropyLoss(ignore_index=-1)(seq_relationship_score.view(-1, 2).float(),
                                                     next_sentence_label.view(-1))
        return seq_relationship_score


class BertForSequenceClassification(BertPreTrainedModel):
    def __init__(self, config, num_labels):
        super().__init__(config)
        self.num_labels = num_labels
        self.bert = BertModel(config)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.classifier = nn.Linear(config.hidden_size, num_labels)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None, checkpoint_activations=False):
        _, pooled_output = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)
        logits = self.classifier(self.dropout(pooled_output))
        if labels is not None:
            return CrossEntropyLoss()(logits.view(-1, self.num_labels).float(), labels.view(-1))
        return logits


class BertForMultipleChoice(BertPreTrainedModel):
    def __init__(self, config, num_choices):
        super().__init__(config)
        self.num_choices = num_choices
        self.bert = BertModel(config)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.classifier = nn.Linear(config.hidden_size, 1)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None, checkpoint_activations=False):
        flat_input_ids = input_ids.reshape(-1, input_ids.size(-1))
        flat_token_type_ids = token_type_ids.reshape(-1, token_type_ids.size(-1))
        flat_attention_mask = attention_mask.reshape(-1, attention_mask.size(-1))
        _, pooled_output = self.bert(flat_input_ids, flat_token_type_ids, flat_attention_mask,
                                     output_all_encoded_layers=False)
        logits = self.classifier(self.dropout(pooled_output))
        reshaped_logits = logits.view(-1, self.num_choices)
        if labels is not None:
            return CrossEntropyLoss()(reshaped_logits.float(), labels)
        return reshaped_logits


class BertForTokenClassification(BertPreTrainedModel):
    def __init__(self, config, num_labels):
        super().__init__(config)
        self.num_labels = num_labels
        self.bert = BertModel(config)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.classifier = nn.Linear(config.hidden_size, num_labels)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None, checkpoint_activations=False):
        sequence_output, _ = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)
        logits = self.classifier(self.dropout(sequence_output))
        if labels is not None:
            loss_fct = CrossEntropyLoss()
            if attention_mask is not None:
                active = attention_mask.view(-1) == 1
                return loss_fct(logits.view(-1, self.num_labels)[active].float(), labels.view(-1)[active])
            return loss_fct(logits.view(-1, self.num_labels).float(), labels.view(-1))
        return logits


class BertForQuestionAnswering(BertPreTrainedModel):
    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)
        self.qa_outputs = nn.Linear(config.hidden_size, 2)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, start_positions=None, end_positions=None,
                checkpoint_activations=False):
        sequence_output, _ = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)
        logits = self.qa_outputs(sequence_output)
        start_logits, end_logits = logits.split(1, dim=-1)
        start_logits, end_logits = start_logits.squeeze(-1), end_logits.squeeze(-1)
        if start_positions is not None and end_positions is not None:
            if len(start_positions.size()) > 1:
                start_positions = start_positions.squeeze(-1)
            if len(end_positions.size()) > 1:
                end_positions = end_positions.squeeze(-1)
            ignored_index = start_logits.size(1)
            start_positions = start_positions.clamp(0, ignored_index)
            end_positions = end_positions.clamp(0, ignored_index)
            loss_fct = CrossEntropyLoss(ignore_index=ignored_index)
            return (loss_fct(start_logits.float(), start_positions) + loss_fct(end_logits.float(), end_positions)) / 2
        return start_logits, end_logits
