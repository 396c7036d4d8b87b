"""T5 / FLAN-T5 encoder-decoder (the RAG lab's generator).

Reference: ``AutoModelForSeq2SeqLM.from_pretrained("google/flan-t5-small")`` +
``generate(max_new_tokens=64)`` in `labs/ragging/rag_example.py:239-270`
("FLAN-T5 gated-GELU").  HF-compatible parameter names
(``shared``, ``encoder.block.{i}.layer.0.SelfAttention.{q,k,v,o}``,
``...relative_attention_bias``, ``layer.1.DenseReluDense.{wi_0,wi_1,wo}``,
``decoder.block.{i}.layer.1.EncDecAttention``, ``lm_head``) so a local
checkpoint loads with ``mift.models.load_hf_weights``.

Architecture (T5 v1.1 / FLAN): RMS LayerNorm (no mean, no bias, fp32),
unscaled dot-product attention plus a learned relative-position bias shared
by all layers of a stack (bidirectional buckets in the encoder, causal in the
decoder, 32 buckets up to distance 128), gated-GELU FFN (gelu_new(wi_0 x) ⊙
wi_1 x), untied LM head.  Greedy decoding keeps a per-layer self-attention
KV cache and precomputes every layer's cross-attention K/V once.

Runs on the autograd path (ATen → hipBLASLt/SDPA on MI355X): a 77 M-parameter
teaching demo, not a kernel target.
"""
import math
from dataclasses import dataclass, asdict

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import reference as ref
from .layers import Embedding, Linear, init_normal_


@dataclass
class T5Config:
    vocab_size: int = 32128
    d_model: int = 512
    d_kv: int = 64
    d_ff: int = 1024
    num_layers: int = 8
    num_decoder_layers: int = 8
    num_heads: int = 6
    relative_attention_num_buckets: int = 32
    relative_attention_max_distance: int = 128
    dropout_rate: float = 0.1
    layer_norm_epsilon: float = 1e-6
    feed_forward_proj: str = "gated-gelu"
    tie_word_embeddings: bool = False
    pad_token_id: int = 0
    eos_token_id: int = 1
    decoder_start_token_id: int = 0
    initializer_factor: float = 1.0
    model_type: str = "t5"

    @staticmethod
    def preset(name):
        n = name.split("/")[-1].lower()
        if n == "flan-t5-small":
            return T5Config()
        if n == "flan-t5-base":
            return T5Config(d_model=768, d_ff=2048, num_layers=12, num_decoder_layers=12, num_heads=12)
        if n in ("t5-tiny", "flan-t5-tiny"):
            return T5Config(vocab_size=512, d_model=64, d_kv=16, d_ff=128, num_layers=2, num_decoder_layers=2,
                            num_heads=4)
        raise ValueError(f"unknown T5 preset {name}")

    def to_hf_dict(self):
        d = asdict(self)
        d.update({"architectures": ["T5ForConditionalGeneration"], "is_encoder_decoder": True,
                  "dense_act_fn": "gelu_new", "is_gated_act": True})
        return d


class T5LayerNorm(nn.Module):
    def __init__(self, d, eps=1e-6, dtype=None, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d, dtype=dtype, device=device))
        self.eps = eps

    def forward(self, x):
        var = x.float().pow(2).mean(-1, keepdim=True)
        y = x.float() * torch.rsqrt(var + self.eps)
        return self.weight * y.to(self.weight.dtype)


def relative_position_bucket(rel, bidirectional, num_buckets, max_distance):
    """HF T5 bucketing of (key - query) offsets."""
    buckets = torch.zeros_like(rel)
    if bidirectional:
        num_buckets //= 2
        buckets = buckets + (rel > 0).long() * num_buckets
        rel = rel.abs()
    else:
        rel = -torch.clamp(rel, max=0)
    max_exact = num_buckets // 2
    small = rel < max_exact
    large = max_exact + (torch.log(rel.float().clamp(min=1) / max_exact) / math.log(max_distance / max_exact)
                         * (num_buckets - max_exact)).long()
    large = torch.clamp(large, max=num_buckets - 1)
    return buckets + torch.where(small, rel, large)


class T5Attention(nn.Module):
    def __init__(self, c: T5Config, causal, has_bias, dtype=None, device=None):
        super().__init__()
        inner = c.num_heads * c.d_kv
        self.c, self.causal, self.has_bias = c, causal, has_bias
        self.q = Linear(c.d_model, inner, bias=False, dtype=dtype, device=device)
        self.k = Linear(c.d_model, inner, bias=False, dtype=dtype, device=device)
        self.v = Linear(c.d_model, inner, bias=False, dtype=dtype, device=device)
        self.o = Linear(inner, c.d_model, bias=False, dtype=dtype, device=device)
        if has_bias:
            self.relative_attention_bias = Embedding(c.relative_attention_num_buckets, c.num_heads, dtype=dtype,
                                                     device=device)

    def position_bias(self, q_pos, k_len, device):
        """[1, H, len(q_pos), k_len] for query positions q_pos (1-D tensor)."""
        rel = torch.arange(k_len, device=device)[None, :] - q_pos[:, None]
        b = relative_position_bucket(rel, not self.causal, self.c.relative_attention_num_buckets,
                                     self.c.relative_attention_max_distance)
        return self.relative_attention_bias(b).permute(2, 0, 1)[None]

    def split(self, x):
        B, S, _ = x.shape
        return x.view(B, S, self.c.num_heads, self.c.d_kv).transpose(1, 2)

    def forward(self, x, kv=None, bias=None, mask=None, cache=None):
        """x [B,Sq,d]; kv: precomputed (k, v) [B,H,Sk,dk] or None (self-attention on x);
        cache: dict holding/receiving the self-attention k/v (decoding)."""
        q = self.split(self.q(x))
        if kv is None:
            k, v = self.split(self.k(x)), self.split(self.v(x))
            if cache is not None:
                if "k" in cache:
                    k, v = torch.cat([cache["k"], k], 2), torch.cat([cache["v"], v], 2)
                cache["k"], cache["v"] = k, v
        else:
            k, v = kv
        s = q.float() @ k.float().transpose(-1, -2)
        if bias is not None:
            s = s + bias
        if mask is not None:
            s = s.masked_fill(~mask, float("-inf"))
        p = torch.softmax(s, -1).to(q.dtype)
        p = F.dropout(p, self.c.dropout_rate, self.training)
        o = (p @ v).transpose(1, 2).reshape(x.shape[0], x.shape[1], -1)
        return self.o(o)


class _Sub(nn.Module):
    """One ``layer.{j}`` entry: LN + sublayer (HF T5LayerSelfAttention / CrossAttention / LayerFF)."""

    def __init__(self, c, kind, causal=False, has_bias=False, dtype=None, device=None):
        super().__init__()
        self.kind = kind
        if kind == "self":
            self.SelfAttention = T5Attention(c, causal, has_bias, dtype, device)
        elif kind == "cross":
            self.EncDecAttention = T5Attention(c, False, False, dtype, device)
        else:
            self.DenseReluDense = nn.Module()
            self.DenseReluDense.wi_0 = Linear(c.d_model, c.d_ff, bias=False, dtype=dtype, device=device)
            self.DenseReluDense.wi_1 = Linear(c.d_model, c.d_ff, bias=False, dtype=dtype, device=device)
            self.DenseReluDense.wo = Linear(c.d_ff, c.d_model, bias=False, dtype=dtype, device=device)
        self.layer_norm = T5LayerNorm(c.d_model, c.layer_norm_epsilon, dtype, device)
        self.p = c.dropout_rate

    def ff(self, x):
        d = self.DenseReluDense
        h = ref.gelu_new(d.wi_0(x)) * d.wi_1(x)
        return d.wo(F.dropout(h, self.p, self.training))


class T5Block(nn.Module):
    def __init__(self, c, decoder, first, dtype=None, device=None):
        super().__init__()
        subs = [_Sub(c, "self", causal=decoder, has_bias=first, dtype=dtype, device=device)]
        if decoder:
            subs.append(_Sub(c, "cross", dtype=dtype, device=device))
        subs.append(_Sub(c, "ff", dtype=dtype, device=device))
        self.layer = nn.ModuleList(subs)
        self.decoder = decoder

    def forward(self, h, self_bias, self_mask, cross_kv=None, cross_mask=None, cache=None):
        p, tr = self.layer[0].p, self.training
        s = self.layer[0]
        h = h + F.dropout(s.SelfAttention(s.layer_norm(h), bias=self_bias, mask=self_mask, cache=cache), p, tr)
        if self.decoder:
            x = self.layer[1]
            h = h + F.dropout(x.EncDecAttention(x.layer_norm(h), kv=cross_kv, mask=cross_mask), p, tr)
        f = self.layer[-1]
        return h + F.dropout(f.ff(f.layer_norm(h)), p, tr)


class T5Stack(nn.Module):
    def __init__(self, c, n, decoder, dtype=None, device=None):
        super().__init__()
        self.block = nn.ModuleList([T5Block(c, decoder, i == 0, dtype, device) for i in range(n)])
        self.final_layer_norm = T5LayerNorm(c.d_model, c.layer_norm_epsilon, dtype, device)
        self.decoder = decoder

    def rel_bias(self):
        return self.block[0].layer[0].SelfAttention


class T5ForConditionalGeneration(nn.Module):
    def __init__(self, cfg: T5Config, dtype=torch.float32, device=None):
        super().__init__()
        self.config = c = cfg
        self.shared = Embedding(c.vocab_size, c.d_model, dtype=dtype, device=device)
        self.encoder = T5Stack(c, c.num_layers, False, dtype, device)
        self.decoder = T5Stack(c, c.num_decoder_layers, True, dtype, device)
        if not c.tie_word_embeddings:
            self.lm_head = Linear(c.d_model, c.vocab_size, bias=False, dtype=dtype, device=device)

    def init_weights(self, seed=0):
        init_normal_(self, 0.05, seed=seed)
        return self

    # ---- pieces ----
    def encode(self, input_ids, attention_mask=None):
        c = self.config
        B, S = input_ids.shape
        h = F.dropout(self.shared(input_ids), c.dropout_rate, self.training)
        att = self.encoder.rel_bias()
        bias = att.position_bias(torch.arange(S, device=h.device), S, h.device)
        mask = attention_mask.bool()[:, None, None, :] if attention_mask is not None else None
        for blk in self.encoder.block:
            h = blk(h, bias, mask)
        return F.dropout(self.encoder.final_layer_norm(h), c.dropout_rate, self.training)

    def cross_kv(self, enc):
        out = []
        for blk in self.decoder.block:
            a = blk.layer[1].EncDecAttention
            out.append((a.split(a.k(enc)), a.split(a.v(enc))))
        return out

    def decode(self, dec_ids, enc, enc_mask, caches=None, start=0, ckv=None):
        c = self.config
        B, T = dec_ids.shape
        h = F.dropout(self.shared(dec_ids), c.dropout_rate, self.training)
        att = self.decoder.rel_bias()
        k_len = start + T
        q_pos = torch.arange(start, start + T, device=h.device)
        bias = att.position_bias(q_pos, k_len, h.device)
        causal = (torch.arange(k_len, device=h.device)[None, :] <= q_pos[:, None])[None, None]
        cmask = enc_mask.bool()[:, None, None, :] if enc_mask is not None else None
        ckv = ckv if ckv is not None else self.cross_kv(enc)
        for i, blk in enumerate(self.decoder.block):
            h = blk(h, bias, causal, cross_kv=ckv[i], cross_mask=cmask, cache=caches[i] if caches else None)
        h = F.dropout(self.decoder.final_layer_norm(h), c.dropout_rate, self.training)
        if c.tie_word_embeddings:
            return (h * c.d_model ** -0.5) @ self.shared.weight.t()
        return self.lm_head(h)

    def shift_right(self, labels):
        c = self.config
        d = torch.full_like(labels, c.pad_token_id)
        d[:, 0] = c.decoder_start_token_id
        d[:, 1:] = labels[:, :-1]
        return d.masked_fill(d == -100, c.pad_token_id)

    def forward(self, input_ids=None, attention_mask=None, labels=None, decoder_input_ids=None, reduction="mean",
                **_):
        enc = self.encode(input_ids, attention_mask)
        if decoder_input_ids is None:
            decoder_input_ids = self.shift_right(labels)
        logits = self.decode(decoder_input_ids, enc, attention_mask)
        out = {"logits": logits}
        if labels is not None:
            out["loss"] = F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), labels.reshape(-1),
                                          ignore_index=-100, reduction=reduction)
        return out

    @torch.no_grad()
    def generate(self, input_ids, attention_mask=None, max_new_tokens=64, eos_token_id=None):
        """Greedy decoding with a self-attention KV cache (HF semantics: starts from
        decoder_start_token_id, finished rows emit pad)."""
        c = self.config
        eos = c.eos_token_id if eos_token_id is None else eos_token_id
        was = self.training
        self.eval()
        enc = self.encode(input_ids, attention_mask)
        ckv = self.cross_kv(enc)
        B = input_ids.shape[0]
        caches = [dict() for _ in self.decoder.block]
        cur = torch.full((B, 1), c.decoder_start_token_id, dtype=torch.long, device=input_ids.device)
        out = [cur]
        done = torch.zeros(B, dtype=torch.bool, device=input_ids.device)
        for t in range(max_new_tokens):
            logits = self.decode(cur, enc, attention_mask, caches=caches, start=t, ckv=ckv)
            nxt = logits[:, -1].float().argmax(-1)
            nxt = torch.where(done, torch.full_like(nxt, c.pad_token_id), nxt)
            out.append(nxt[:, None])
            done = done | (nxt == eos)
            cur = nxt[:, None]
            if bool(done.all()):
                break
        self.train(was)
        return torch.cat(out, 1)
