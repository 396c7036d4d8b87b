"""RoBERTa and DistilBERT sequence classifiers (the remaining lab encoders).

Reference labs: ``distilroberta-base`` on AG-News
(`labs/simple_model/train_simple.py:104-110`) and ``distilbert-base-uncased``
transfer learning (`labs/transfer_learning/transfer.py:57-60`), both through
``AutoModelForSequenceClassification``.  HF parameter names are kept
(``roberta.encoder.layer.{i}...`` / ``classifier.dense|out_proj``;
``distilbert.transformer.layer.{i}.attention.q_lin`` ... ``pre_classifier``)
so local checkpoints load with ``mift.models.load_hf_weights``.

Both are post-LN encoders with GELU FFNs and key-padding masks; they reuse
BERT's layer (``mift.models.bert.BertLayer``, HF's own layer is shared the
same way) where names coincide.  Full fine-tuning on the autograd path
(ATen → hipBLASLt/SDPA) like the tiny BERT: lab models, not kernel targets.
"""
import json
import os
from dataclasses import dataclass, asdict

import torch
import torch.nn as nn
import torch.nn.functional as F

from .bert import BertConfig, BertLayer
from .layers import Embedding, LayerNorm, Linear, init_normal_


# ---------------------------------------------------------------- RoBERTa
@dataclass
class RobertaConfig(BertConfig):
    vocab_size: int = 50265
    hidden_size: int = 768
    num_hidden_layers: int = 6
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 514
    type_vocab_size: int = 1
    layer_norm_eps: float = 1e-5
    pad_token_id: int = 1
    model_type: str = "roberta"

    @staticmethod
    def preset(name, num_labels=4):
        n = name.split("/")[-1].lower()
        if n == "distilroberta-base":
            return RobertaConfig(num_labels=num_labels)
        if n == "roberta-base":
            return RobertaConfig(num_hidden_layers=12, num_labels=num_labels)
        if n == "roberta-tiny":
            return RobertaConfig(vocab_size=300, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                 intermediate_size=128, max_position_embeddings=130, num_labels=num_labels)
        raise ValueError(name)

    def to_hf_dict(self):
        d = asdict(self)
        d.update({"architectures": ["RobertaForSequenceClassification"], "hidden_act": "gelu",
                  "id2label": {str(i): f"LABEL_{i}" for i in range(self.num_labels)},
                  "label2id": {f"LABEL_{i}": i for i in range(self.num_labels)}})
        return d


class RobertaForSequenceClassification(nn.Module):
    def __init__(self, cfg: RobertaConfig, dtype=torch.float32, device=None):
        super().__init__()
        self.config = c = cfg
        self.roberta = nn.Module()
        e = self.roberta.embeddings = nn.Module()
        e.word_embeddings = Embedding(c.vocab_size, c.hidden_size, dtype=dtype, device=device)
        e.position_embeddings = Embedding(c.max_position_embeddings, c.hidden_size, dtype=dtype, device=device)
        e.token_type_embeddings = Embedding(c.type_vocab_size, c.hidden_size, dtype=dtype, device=device)
        e.LayerNorm = LayerNorm(c.hidden_size, c.layer_norm_eps, dtype=dtype, device=device)
        self.roberta.encoder = nn.Module()
        self.roberta.encoder.layer = nn.ModuleList([BertLayer(c, dtype, device) for _ in range(c.num_hidden_layers)])
        self.classifier = nn.Module()
        self.classifier.dense = Linear(c.hidden_size, c.hidden_size, dtype=dtype, device=device)
        self.classifier.out_proj = Linear(c.hidden_size, c.num_labels, dtype=dtype, device=device)
        self.micro_step = 0

    def init_weights(self, seed=0):
        init_normal_(self, self.config.initializer_range, seed=seed)
        return self

    def next_micro_step(self):
        self.micro_step += 1

    @staticmethod
    def count_targets(labels):
        return int((labels != -100).sum())

    def forward(self, input_ids=None, attention_mask=None, labels=None, reduction="mean", **_):
        c = self.config
        e = self.roberta.embeddings
        tok_mask = (input_ids != c.pad_token_id).long()
        pos = torch.cumsum(tok_mask, 1) * tok_mask + c.pad_token_id  # HF create_position_ids_from_input_ids
        h = e.word_embeddings(input_ids) + e.position_embeddings(pos) + \
            e.token_type_embeddings(torch.zeros_like(input_ids))
        h = F.dropout(e.LayerNorm(h), c.hidden_dropout_prob, self.training)
        km = attention_mask.bool()[:, None, None, :] if attention_mask is not None else None
        for layer in self.roberta.encoder.layer:
            h = layer(h, km)
        x = F.dropout(h[:, 0], c.hidden_dropout_prob, self.training)
        x = F.dropout(torch.tanh(self.classifier.dense(x)), c.hidden_dropout_prob, self.training)
        logits = self.classifier.out_proj(x)
        out = {"logits": logits}
        if labels is not None:
            out["loss"] = F.cross_entropy(logits.float(), labels, ignore_index=-100, reduction=reduction)
        return out

    def save_pretrained(self, d):
        _save(self, d)


# ---------------------------------------------------------------- DistilBERT
@dataclass
class DistilBertConfig:
    vocab_size: int = 30522
    dim: int = 768
    n_layers: int = 6
    n_heads: int = 12
    hidden_dim: int = 3072
    max_position_embeddings: int = 512
    dropout: float = 0.1
    attention_dropout: float = 0.1
    seq_classif_dropout: float = 0.2
    initializer_range: float = 0.02
    num_labels: int = 2
    pad_token_id: int = 0
    model_type: str = "distilbert"

    @staticmethod
    def preset(name, num_labels=2):
        n = name.split("/")[-1].lower()
        if n in ("distilbert-base-uncased", "distilbert-base-cased"):
            return DistilBertConfig(num_labels=num_labels)
        if n == "distilbert-tiny":
            return DistilBertConfig(vocab_size=300, dim=64, n_layers=2, n_heads=2, hidden_dim=128,
                                    max_position_embeddings=128, num_labels=num_labels)
        raise ValueError(name)

    def to_hf_dict(self):
        d = asdict(self)
        d.update({"architectures": ["DistilBertForSequenceClassification"], "activation": "gelu",
                  "id2label": {str(i): f"LABEL_{i}" for i in range(self.num_labels)},
                  "label2id": {f"LABEL_{i}": i for i in range(self.num_labels)}})
        return d


class _DBLayer(nn.Module):
    def __init__(self, c, dtype=None, device=None):
        super().__init__()
        self.c = c
        self.attention = nn.Module()
        for n in ("q_lin", "k_lin", "v_lin", "out_lin"):
            setattr(self.attention, n, Linear(c.dim, c.dim, dtype=dtype, device=device))
        self.sa_layer_norm = LayerNorm(c.dim, 1e-12, dtype=dtype, device=device)
        self.ffn = nn.Module()
        self.ffn.lin1 = Linear(c.dim, c.hidden_dim, dtype=dtype, device=device)
        self.ffn.lin2 = Linear(c.hidden_dim, c.dim, dtype=dtype, device=device)
        self.output_layer_norm = LayerNorm(c.dim, 1e-12, dtype=dtype, device=device)

    def forward(self, h, km):
        c, (B, S, d) = self.c, h.shape
        H, hd = c.n_heads, c.dim // c.n_heads
        a = self.attention
        q = a.q_lin(h).view(B, S, H, hd).transpose(1, 2)
        k = a.k_lin(h).view(B, S, H, hd).transpose(1, 2)
        v = a.v_lin(h).view(B, S, H, hd).transpose(1, 2)
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=km,
                                           dropout_p=c.attention_dropout if self.training else 0.0)
        h = self.sa_layer_norm(h + a.out_lin(o.transpose(1, 2).reshape(B, S, d)))
        f = F.dropout(self.ffn.lin2(F.gelu(self.ffn.lin1(h))), c.dropout, self.training)
        return self.output_layer_norm(h + f)


class DistilBertForSequenceClassification(nn.Module):
    def __init__(self, cfg: DistilBertConfig, dtype=torch.float32, device=None):
        super().__init__()
        self.config = c = cfg
        self.distilbert = nn.Module()
        e = self.distilbert.embeddings = nn.Module()
        e.word_embeddings = Embedding(c.vocab_size, c.dim, dtype=dtype, device=device)
        e.position_embeddings = Embedding(c.max_position_embeddings, c.dim, dtype=dtype, device=device)
        e.LayerNorm = LayerNorm(c.dim, 1e-12, dtype=dtype, device=device)
        self.distilbert.transformer = nn.Module()
        self.distilbert.transformer.layer = nn.ModuleList([_DBLayer(c, dtype, device) for _ in range(c.n_layers)])
        self.pre_classifier = Linear(c.dim, c.dim, dtype=dtype, device=device)
        self.classifier = Linear(c.dim, c.num_labels, dtype=dtype, device=device)
        self.micro_step = 0

    def init_weights(self, seed=0):
        init_normal_(self, self.config.initializer_range, seed=seed)
        return self

    def next_micro_step(self):
        self.micro_step += 1

    @staticmethod
    def count_targets(labels):
        return int((labels != -100).sum())

    def forward(self, input_ids=None, attention_mask=None, labels=None, reduction="mean", **_):
        c = self.config
        e = self.distilbert.embeddings
        S = input_ids.shape[1]
        h = e.word_embeddings(input_ids) + e.position_embeddings(torch.arange(S, device=input_ids.device))[None]
        h = F.dropout(e.LayerNorm(h), c.dropout, self.training)
        km = attention_mask.bool()[:, None, None, :] if attention_mask is not None else None
        for layer in self.distilbert.transformer.layer:
            h = layer(h, km)
        x = F.relu(self.pre_classifier(h[:, 0]))
        logits = self.classifier(F.dropout(x, c.seq_classif_dropout, self.training))
        out = {"logits": logits}
        if labels is not None:
            out["loss"] = F.cross_entropy(logits.float(), labels, ignore_index=-100, reduction=reduction)
        return out

    def save_pretrained(self, d):
        _save(self, d)


def _save(model, d):
    from safetensors.torch import save_file
    os.makedirs(d, exist_ok=True)
    save_file({k: v.detach().contiguous().cpu() for k, v in model.state_dict().items()},
              os.path.join(d, "model.safetensors"), metadata={"format": "pt"})
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(model.config.to_hf_dict(), f, indent=2)


def build_classifier(name, num_labels, dtype=torch.float32, device=None, seed=0, weights=None):
    """Reference model id -> our classifier (random init unless a local HF checkpoint dir is given)."""
    n = name.lower()
    if "distilbert" in n:
        m = DistilBertForSequenceClassification(DistilBertConfig.preset(name, num_labels), dtype, device)
    elif "roberta" in n:
        m = RobertaForSequenceClassification(RobertaConfig.preset(name, num_labels), dtype, device)
    else:
        from .bert import BertForSequenceClassification
        m = BertForSequenceClassification(BertConfig.tiny(num_labels=num_labels), dtype, device)
    m.init_weights(seed)
    if weights:
        from . import load_hf_weights
        load_hf_weights(m, weights)
    return m
