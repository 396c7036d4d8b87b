"""GPT-2 family (distilgpt2 = 6 layers) causal LM.

Architecture parity: HF ``GPT2LMHeadModel`` as used by the reference
(`Cluster/Project 1 - Fine Tuning Distilgpt2/finetune_lora_distilgpt2.py:80-92`,
spec in README.md:52-61 / SURVEY Appendix C): pre-LN blocks, fused qkv
``c_attn`` (Conv1D [in,out]), ``gelu_new`` MLP, learned positions, dropout
0.1 (embd/attn/resid), LN eps 1e-5, LM head tied to ``wte``.

Two execution paths over the same parameters:
  * reference path (this file) — plain torch autograd, any device; the
    CPU/gloo plumbing configuration and the numerics oracle;
  * fused HIP path (``mift.models.gpt2_fused``) — block-level autograd
    Functions over the gfx950 kernels; used for GPU tensors.
"""
from dataclasses import dataclass, asdict

import torch
import torch.nn as nn

from ..ops import reference as ref
from .base import CausalLMBase, normalize_chunks, ref_lm_loss
from .layers import Embedding, LayerNorm, Linear, dropout_seed, init_normal_, padded_vocab, seed_for


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 6
    n_head: int = 12
    n_inner: int = 3072
    layer_norm_epsilon: float = 1e-5
    embd_pdrop: float = 0.1
    attn_pdrop: float = 0.1
    resid_pdrop: float = 0.1
    initializer_range: float = 0.02
    bos_token_id: int = 50256
    eos_token_id: int = 50256
    pad_token_id: int = 50256
    model_type: str = "gpt2"

    @staticmethod
    def preset(name: str) -> "GPT2Config":
        name = name.split("/")[-1].lower()
        if name in ("distilgpt2", "distilgpt2-lora"):
            return GPT2Config(n_layer=6)
        if name == "gpt2":
            return GPT2Config(n_layer=12)
        if name == "gpt2-medium":
            return GPT2Config(n_layer=24, n_embd=1024, n_head=16, n_inner=4096)
        if name in ("gpt2-tiny", "tiny-gpt2"):
            return GPT2Config(n_layer=2, n_embd=64, n_head=2, n_inner=256, vocab_size=1000, n_positions=128)
        raise ValueError(f"unknown GPT-2 preset {name}")

    def num_layers(self):
        return self.n_layer

    def to_hf_dict(self):
        d = asdict(self)
        d.update({"architectures": ["GPT2LMHeadModel"], "activation_function": "gelu_new",
                  "n_ctx": self.n_positions, "tie_word_embeddings": True})
        return d


class GPT2Attention(nn.Module):
    def __init__(self, cfg: GPT2Config, dtype=None, device=None):
        super().__init__()
        self.n_head = cfg.n_head
        self.head_dim = cfg.n_embd // cfg.n_head
        self.c_attn = Linear(cfg.n_embd, 3 * cfg.n_embd, conv1d=True, dtype=dtype, device=device)
        self.c_proj = Linear(cfg.n_embd, cfg.n_embd, conv1d=True, dtype=dtype, device=device)


class GPT2MLP(nn.Module):
    def __init__(self, cfg: GPT2Config, dtype=None, device=None):
        super().__init__()
        self.c_fc = Linear(cfg.n_embd, cfg.n_inner, conv1d=True, dtype=dtype, device=device)
        self.c_proj = Linear(cfg.n_inner, cfg.n_embd, conv1d=True, dtype=dtype, device=device)


class GPT2Block(nn.Module):
    def __init__(self, cfg: GPT2Config, idx: int, dtype=None, device=None):
        super().__init__()
        self.idx = idx
        self.cfg = cfg
        self.ln_1 = LayerNorm(cfg.n_embd, cfg.layer_norm_epsilon, dtype=dtype, device=device)
        self.attn = GPT2Attention(cfg, dtype, device)
        self.ln_2 = LayerNorm(cfg.n_embd, cfg.layer_norm_epsilon, dtype=dtype, device=device)
        self.mlp = GPT2MLP(cfg, dtype, device)

    def site_seeds(self, base, step):
        s = 100 + 10 * self.idx
        return {k: dropout_seed(base, step, s + i) for i, k in
                enumerate(["attn", "attn_out", "mlp_out", "lora_attn", "lora_proj", "lora_mlp"])}

    def forward_ref(self, h, seeds, training, key_valid=None, attn=None):
        """h: [B, S, d] (reference path).  ``attn(qkv) -> o`` overrides the attention
        (KV-cache decode / padded prefill in mift.infer.generate)."""
        B, S, d = h.shape
        H, hd = self.attn.n_head, self.attn.head_dim
        cfg = self.cfg
        a = self.ln_1(h)
        qkv = self.attn.c_attn(a, seeds["lora_attn"])
        if attn is not None:
            o = attn(qkv)
        else:
            q, k, v = qkv.split(d, dim=-1)
            q = q.view(B, S, H, hd).transpose(1, 2)
            k = k.view(B, S, H, hd).transpose(1, 2)
            v = v.view(B, S, H, hd).transpose(1, 2)
            o = ref.attention(q, k, v, causal=True, key_padding=key_valid, scale=hd ** -0.5,
                              dropout_p=cfg.attn_pdrop if training else 0.0, seed=seeds["attn"])
            o = o.transpose(1, 2).reshape(B, S, d)
        y = self.attn.c_proj(o, seeds["lora_proj"])
        if training and cfg.resid_pdrop > 0:
            y = ref.dropout(y, cfg.resid_pdrop, seeds["attn_out"])
        h = h + y
        a2 = self.ln_2(h)
        f = ref.gelu_new(self.mlp.c_fc(a2))
        y2 = self.mlp.c_proj(f, seeds["lora_mlp"])
        if training and cfg.resid_pdrop > 0:
            y2 = ref.dropout(y2, cfg.resid_pdrop, seeds["mlp_out"])
        return h + y2

    def forward_fused(self, h, seeds, training, kv_len=None, attn=None):
        """Fused HIP path: LN+c_attn(+LoRA) -> attention -> c_proj(+LoRA)+dropout+residual
        -> LN+c_fc+gelu_new -> c_proj(+LoRA)+dropout+residual (mift.ops.fused)."""
        from ..ops import fused as F
        from ..ops.attention import causal_attention
        cfg = self.cfg
        B, S, d = h.shape
        H, hd = self.attn.n_head, self.attn.head_dim
        link = F.ResidualLink()  # residual grad of h enters the LN backward (no separate add kernel)
        qkv = F.ln_linear(h, self.ln_1, self.attn.c_attn, seeds["lora_attn"], training, link=link)
        if attn is not None:
            o = attn(qkv)
        else:
            o = causal_attention(qkv, B, S, H, hd, scale=hd ** -0.5, dropout_p=cfg.attn_pdrop if training else 0.0,
                                 seed=seeds["attn"], kv_len=kv_len)
        # the MLP's LN backward also runs c_proj's residual-dropout backward + dT (one row pass)
        hand = F.GradHandoff() if training and torch.is_grad_enabled() else None
        h = F.linear_residual(o, h, self.attn.c_proj, cfg.resid_pdrop, seeds["attn_out"], seeds["lora_proj"],
                              training, link=link, handoff=hand)
        return F.mlp(h, self.ln_2, self.mlp.c_fc, self.mlp.c_proj, act=1, p=cfg.resid_pdrop, seed=seeds["mlp_out"],
                     seed_l1=0, seed_l2=seeds["lora_mlp"], training=training, handoff=hand)


class GPT2LMHeadModel(CausalLMBase):
    """HF-compatible GPT-2 LM.  ``forward(input_ids, attention_mask, labels)``."""

    def __init__(self, cfg: GPT2Config, dtype=torch.float32, device=None, layer_range=None,
                 has_embed=True, has_head=True):
        super().__init__()
        self.config = cfg
        self.dtype_ = dtype
        n = cfg.n_layer
        self.layer_range, self.chunk_ranges, member = normalize_chunks(layer_range, n)
        self.has_embed, self.has_head = has_embed, has_head
        self.vocab_padded = padded_vocab(cfg.vocab_size)
        self.transformer = nn.Module()
        if has_embed or has_head:
            self.transformer.wte = Embedding(cfg.vocab_size, cfg.n_embd, dtype=dtype, device=device)
        if has_embed:
            self.transformer.wpe = Embedding(cfg.n_positions, cfg.n_embd, dtype=dtype, device=device)
        self.transformer.h = nn.ModuleList(
            [GPT2Block(cfg, i, dtype, device) if member[i] else nn.Identity() for i in range(n)])
        if has_head:
            self.transformer.ln_f = LayerNorm(cfg.n_embd, cfg.layer_norm_epsilon, dtype=dtype, device=device)
        self._init_runtime(self.vocab_padded)

    # ---- init / misc ----
    def init_weights(self, seed=0):
        std = self.config.initializer_range
        init_normal_(self, std, proj_std=std / (2 * self.config.n_layer) ** 0.5, seed=seed)
        return self

    def all_blocks(self):
        return [b for b in self.transformer.h if isinstance(b, GPT2Block)]

    def tied_embedding(self):
        return self.transformer.wte.weight

    def embedding_tables(self):
        return self.transformer.wte, self.transformer.wpe

    def final_norm(self):
        return self.transformer.ln_f

    # ---- reference path pieces ----
    def embed_ref(self, input_ids, attention_mask=None):
        B, S = input_ids.shape
        pos = torch.arange(S, device=input_ids.device)
        h = self.transformer.wte(input_ids) + self.transformer.wpe(pos)[None]
        if self.training and self.config.embd_pdrop > 0:
            h = ref.dropout(h, self.config.embd_pdrop, self.embed_seed())
        return h

    def head_ref(self, h, labels, reduction="mean"):
        h = self.transformer.ln_f(h)
        logits = h @ self.transformer.wte.weight.t()
        if labels is None:
            return None, logits
        return ref_lm_loss(logits, labels, -100, reduction), logits

    def forward(self, input_ids=None, attention_mask=None, labels=None, hidden_states=None, reduction="mean",
                return_logits=True):
        ref_in = input_ids if input_ids is not None else hidden_states
        if self._use_fused(ref_in):
            from .gpt2_fused import fused_forward
            return fused_forward(self, input_ids, attention_mask, labels, hidden_states, reduction, return_logits)
        key_valid = None
        h = self.embed_ref(input_ids, attention_mask) if self.embed_here else hidden_states
        for blk in self.blocks():
            seeds = blk.site_seeds(self.seed, self.micro_step)
            if self.recompute and self.training:
                h = torch.utils.checkpoint.checkpoint(blk.forward_ref, h, seeds, self.training, key_valid,
                                                      use_reentrant=False)
            else:
                h = blk.forward_ref(h, seeds, self.training, key_valid)
        if not self.head_here:
            return {"hidden_states": h}
        loss, logits = self.head_ref(h, labels, reduction)
        return {"loss": loss, "logits": logits if return_logits else None}
