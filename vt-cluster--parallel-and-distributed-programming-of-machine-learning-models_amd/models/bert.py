"""BERT encoder + sequence-classification head (the tiny-lab model).

Reference: ``BertForSequenceClassification(BertConfig(hidden=64, layers=2,
heads=2, intermediate=256, max_pos=256))`` with the
``google/bert_uncased_L-2_H-128_A-2`` WordPiece vocab, fully fine-tuned on
AG-News (`labs/tiny/train_tiny.py:89-99`, `:143-146`).
Parameter names are HF's (``bert.embeddings.word_embeddings.weight``,
``bert.encoder.layer.{i}.attention.self.query.weight``, ...,
``bert.pooler.dense``, ``classifier``) so ``save_pretrained`` output loads in
``transformers`` and vice versa.

Architecture: post-LN encoder (h = LN(h + drop(Attn(h))); h = LN(h +
drop(FFN(h)))), GELU (erf), LN eps 1e-12, padding-key attention mask, tanh
pooler over [CLS], dropout 0.1 everywhere.  The lab trains ALL weights, so
this model runs on the autograd path (ATen → hipBLASLt GEMMs and the fused
SDPA on MI355X); at 0.5 M parameters it is launch-bound, not a kernel
target ("generic GEMM path is enough").
"""
import json
import os
from dataclasses import dataclass, asdict

import torch
import torch.nn as nn
import torch.nn.functional as F

from .layers import Embedding, LayerNorm, Linear, init_normal_


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 64
    num_hidden_layers: int = 2
    num_attention_heads: int = 2
    intermediate_size: int = 256
    max_position_embeddings: int = 256
    type_vocab_size: int = 2
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02
    num_labels: int = 4
    pad_token_id: int = 0
    model_type: str = "bert"

    @staticmethod
    def tiny(vocab_size=30522, num_labels=4):
        """`labs/tiny/train_tiny.py:89-99`."""
        return BertConfig(vocab_size=vocab_size, num_labels=num_labels)

    def to_hf_dict(self):
        d = asdict(self)
        d.update({"architectures": ["BertForSequenceClassification"], "hidden_act": "gelu",
                  "id2label": {str(i): f"LABEL_{i}" for i in range(self.num_labels)},
                  "label2id": {f"LABEL_{i}": i for i in range(self.num_labels)},
                  "position_embedding_type": "absolute"})
        return d

    @staticmethod
    def from_hf_dict(d):
        keys = BertConfig.__dataclass_fields__.keys()
        c = BertConfig(**{k: v for k, v in d.items() if k in keys})
        if "id2label" in d:
            c.num_labels = len(d["id2label"])
        return c


class _Attn(nn.Module):
    def __init__(self, c, dtype, device):
        super().__init__()
        self.self = nn.Module()
        self.self.query = Linear(c.hidden_size, c.hidden_size, dtype=dtype, device=device)
        self.self.key = Linear(c.hidden_size, c.hidden_size, dtype=dtype, device=device)
        self.self.value = Linear(c.hidden_size, c.hidden_size, dtype=dtype, device=device)
        self.output = nn.Module()
        self.output.dense = Linear(c.hidden_size, c.hidden_size, dtype=dtype, device=device)
        self.output.LayerNorm = LayerNorm(c.hidden_size, c.layer_norm_eps, dtype=dtype, device=device)


class BertLayer(nn.Module):
    def __init__(self, c, dtype=None, device=None):
        super().__init__()
        self.c = c
        self.attention = _Attn(c, dtype, device)
        self.intermediate = nn.Module()
        self.intermediate.dense = Linear(c.hidden_size, c.intermediate_size, dtype=dtype, device=device)
        self.output = nn.Module()
        self.output.dense = Linear(c.intermediate_size, c.hidden_size, dtype=dtype, device=device)
        self.output.LayerNorm = LayerNorm(c.hidden_size, c.layer_norm_eps, dtype=dtype, device=device)

    def forward(self, h, key_mask):
        c, B, S, d = self.c, h.shape[0], h.shape[1], h.shape[2]
        H = c.num_attention_heads
        hd = d // H
        sa = self.attention.self
        q = sa.query(h).view(B, S, H, hd).transpose(1, 2)
        k = sa.key(h).view(B, S, H, hd).transpose(1, 2)
        v = sa.value(h).view(B, S, H, hd).transpose(1, 2)
        p = c.attention_probs_dropout_prob if self.training else 0.0
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=key_mask, dropout_p=p)
        o = o.transpose(1, 2).reshape(B, S, d)
        ao = self.attention.output
        h = ao.LayerNorm(h + F.dropout(ao.dense(o), c.hidden_dropout_prob, self.training))
        f = F.gelu(self.intermediate.dense(h))
        return self.output.LayerNorm(h + F.dropout(self.output.dense(f), c.hidden_dropout_prob, self.training))


class BertForSequenceClassification(nn.Module):
    def __init__(self, cfg: BertConfig, dtype=torch.float32, device=None):
        super().__init__()
        self.config = cfg
        c = cfg
        self.bert = nn.Module()
        e = self.bert.embeddings = nn.Module()
        e.word_embeddings = Embedding(c.vocab_size, c.hidden_size, dtype=dtype, device=device)
        e.position_embeddings = Embedding(c.max_position_embeddings, c.hidden_size, dtype=dtype, device=device)
        e.token_type_embeddings = Embedding(c.type_vocab_size, c.hidden_size, dtype=dtype, device=device)
        e.LayerNorm = LayerNorm(c.hidden_size, c.layer_norm_eps, dtype=dtype, device=device)
        self.bert.encoder = nn.Module()
        self.bert.encoder.layer = nn.ModuleList([BertLayer(c, dtype, device) for _ in range(c.num_hidden_layers)])
        self.bert.pooler = nn.Module()
        self.bert.pooler.dense = Linear(c.hidden_size, c.hidden_size, dtype=dtype, device=device)
        self.classifier = Linear(c.hidden_size, c.num_labels, dtype=dtype, device=device)
        self.micro_step = 0
        self.seed = 0

    def init_weights(self, seed=0):
        init_normal_(self, self.config.initializer_range, seed=seed)
        return self

    # trainer protocol
    def next_micro_step(self):
        self.micro_step += 1

    @staticmethod
    def count_targets(labels):
        return int((labels != -100).sum())

    def forward(self, input_ids=None, attention_mask=None, labels=None, token_type_ids=None, reduction="mean",
                return_logits=True, **_):
        c = self.config
        B, S = input_ids.shape
        e = self.bert.embeddings
        pos = torch.arange(S, device=input_ids.device)[None]
        tt = token_type_ids if token_type_ids is not None else torch.zeros_like(input_ids)
        h = e.word_embeddings(input_ids) + e.position_embeddings(pos) + e.token_type_embeddings(tt)
        h = F.dropout(e.LayerNorm(h), c.hidden_dropout_prob, self.training)
        key_mask = None
        if attention_mask is not None:
            key_mask = attention_mask.bool()[:, None, None, :]
        for layer in self.bert.encoder.layer:
            h = layer(h, key_mask)
        pooled = torch.tanh(self.bert.pooler.dense(h[:, 0]))
        logits = self.classifier(F.dropout(pooled, c.hidden_dropout_prob, self.training))
        out = {"logits": logits}
        if labels is not None:
            out["loss"] = F.cross_entropy(logits.float(), labels, ignore_index=-100, reduction=reduction)
            out["ntokens"] = (labels != -100).sum()
        return out

    # ---- HF-format I/O ----
    def save_pretrained(self, d):
        from safetensors.torch import save_file
        os.makedirs(d, exist_ok=True)
        save_file({k: v.detach().contiguous().cpu() for k, v in self.state_dict().items()},
                  os.path.join(d, "model.safetensors"), metadata={"format": "pt"})
        with open(os.path.join(d, "config.json"), "w") as f:
            json.dump(self.config.to_hf_dict(), f, indent=2)

    @staticmethod
    def from_pretrained(d, dtype=torch.float32, device=None):
        with open(os.path.join(d, "config.json")) as f:
            cfg = BertConfig.from_hf_dict(json.load(f))
        m = BertForSequenceClassification(cfg, dtype=dtype, device=device)
        from . import load_hf_weights
        missing = load_hf_weights(m, d)
        if missing:
            raise KeyError(f"checkpoint {d} lacks {missing[:4]}")
        return m
