"""OPT family (facebook/opt-125m ... opt-6.7b) causal LM.

Architecture parity with HF ``OPTForCausalLM`` as the reference loads it
(`Cluster/Project 2 - Course Project/finetune_lora_opt_pp.py:94-98`; spec in
SURVEY §3.4 / Appendix C): pre-LN decoder layers (``do_layer_norm_before``),
separate ``q_proj/k_proj/v_proj/out_proj`` (nn.Linear [out,in] + bias), ReLU
``fc1``/``fc2`` MLP, learned positions with offset 2 and
``positions = cumsum(mask)·mask - 1`` (HF ``OPTLearnedPositionalEmbedding``),
dropout 0.1 after out_proj and fc2, attention dropout 0, no embedding
dropout, final LayerNorm, LM head tied to ``embed_tokens``.  Parameter names
match HF (``model.decoder.layers.{i}.self_attn.q_proj.weight`` ...) so
checkpoints and PEFT adapters (``base_model.model.model.decoder...``)
interchange.

Stage construction mirrors the reference's ``OPTEmb`` / ``OPTBlk`` /
``OPTHead`` wrappers (`finetune_lora_opt_pp.py:121-153`) but a stage only
ALLOCATES its own layers (``layer_range``, ``has_embed``, ``has_head``): the
reference loads the full fp32 model on every rank and is OOM-killed there
(SURVEY §6).  The pipeline loss head keeps the reference's
``ignore_index=pad_token_id`` option (`:143`), default HF -100.

Execution paths: reference torch autograd (CPU / oracle) and the fused HIP
path (q/k/v as ONE GEMM with a multi-adapter LoRA K-extension — see
``ConcatLinear`` — flash attention at head dim 80/128, ReLU fused into the
fc1 epilogue and its derivative into the fc2 dgrad epilogue).
Not supported: opt-350m's post-LN / project_in/out variant.
"""
from dataclasses import dataclass, asdict

import torch
import torch.nn as nn

from ..ops import reference as ref
from .base import CausalLMBase, chunk_parts, normalize_chunks, ref_lm_loss, shift_labels
from .layers import ConcatLinear, Embedding, LayerNorm, Linear, dropout_seed, init_normal_, padded_vocab, seed_for


@dataclass
class OPTConfig:
    vocab_size: int = 50272
    hidden_size: int = 2560
    num_hidden_layers: int = 32
    ffn_dim: int = 10240
    num_attention_heads: int = 32
    max_position_embeddings: int = 2048
    dropout: float = 0.1
    attention_dropout: float = 0.0
    activation_function: str = "relu"
    do_layer_norm_before: bool = True
    enable_bias: bool = True
    layer_norm_eps: float = 1e-5
    init_std: float = 0.02
    pad_token_id: int = 1
    bos_token_id: int = 2
    eos_token_id: int = 2
    model_type: str = "opt"

    _PRESETS = {
        "opt-125m": (768, 12, 12, 3072),
        "opt-1.3b": (2048, 24, 32, 8192),
        "opt-2.7b": (2560, 32, 32, 10240),
        "opt-6.7b": (4096, 32, 32, 16384),
        "opt-13b": (5120, 40, 40, 20480),
    }

    @staticmethod
    def preset(name: str) -> "OPTConfig":
        n = name.split("/")[-1].lower()
        if n in ("opt-tiny", "tiny-opt"):
            return OPTConfig(vocab_size=1000, hidden_size=64, num_hidden_layers=4, ffn_dim=256,
                             num_attention_heads=2, max_position_embeddings=128)
        if n == "opt-350m":
            raise ValueError("opt-350m (post-LN + project_in/out) is not supported")
        if n not in OPTConfig._PRESETS:
            raise ValueError(f"unknown OPT preset {name}")
        d, L, H, f = OPTConfig._PRESETS[n]
        return OPTConfig(hidden_size=d, num_hidden_layers=L, num_attention_heads=H, ffn_dim=f)

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    def num_layers(self):
        return self.num_hidden_layers

    def to_hf_dict(self):
        d = {k: v for k, v in asdict(self).items()}
        d.update({"architectures": ["OPTForCausalLM"], "word_embed_proj_dim": self.hidden_size,
                  "layerdrop": 0.0, "layer_norm_elementwise_affine": True, "tie_word_embeddings": True,
                  "_remove_final_layer_norm": False})
        return d


class OPTAttention(nn.Module):
    def __init__(self, cfg: OPTConfig, dtype=None, device=None):
        super().__init__()
        d, b = cfg.hidden_size, cfg.enable_bias
        self.n_head, self.head_dim = cfg.num_attention_heads, cfg.head_dim
        self.q_proj = Linear(d, d, bias=b, dtype=dtype, device=device)
        self.k_proj = Linear(d, d, bias=b, dtype=dtype, device=device)
        self.v_proj = Linear(d, d, bias=b, dtype=dtype, device=device)
        self.out_proj = Linear(d, d, bias=b, dtype=dtype, device=device)
        self.__dict__["qkv"] = ConcatLinear([self.q_proj, self.k_proj, self.v_proj])


class OPTDecoderLayer(nn.Module):
    SITES = ["attn", "attn_out", "mlp_out", "lora_attn", "lora_proj", "lora_fc1", "lora_fc2"]

    def __init__(self, cfg: OPTConfig, idx: int, dtype=None, device=None, parts=(True, True)):
        """``parts`` = (attention sub-block, MLP sub-block) this stage holds: a half-layer pipeline
        boundary (models/base.py ``normalize_chunks``) builds only its side's weights and adapters."""
        super().__init__()
        self.idx, self.cfg, self.parts = idx, cfg, tuple(parts)
        d = cfg.hidden_size
        if parts[0]:
            self.self_attn = OPTAttention(cfg, dtype, device)
            self.self_attn_layer_norm = LayerNorm(d, cfg.layer_norm_eps, dtype=dtype, device=device)
        if parts[1]:
            self.fc1 = Linear(d, cfg.ffn_dim, bias=cfg.enable_bias, dtype=dtype, device=device)
            self.fc2 = Linear(cfg.ffn_dim, d, bias=cfg.enable_bias, dtype=dtype, device=device)
            self.final_layer_norm = LayerNorm(d, cfg.layer_norm_eps, dtype=dtype, device=device)

    def site_seeds(self, base, step):
        s = 100 + 10 * self.idx
        return {k: dropout_seed(base, step, s + i) for i, k in enumerate(self.SITES)}

    def forward_ref(self, h, seeds, training, key_valid=None, attn=None, parts=(True, True)):
        """h: [B, S, d] (reference path).  One LoRA-dropout seed for q/k/v (see MultiAdapterOps).
        ``attn(qkv [B,S,3d]) -> o [B,S,d]`` overrides the attention (KV-cache decode).  ``parts``:
        the sub-blocks to run (a half-layer pipeline stage runs one)."""
        cfg = self.cfg
        B, S, d = h.shape
        if parts[0]:
            H, hd = self.self_attn.n_head, self.self_attn.head_dim
            at = self.self_attn
            a = self.self_attn_layer_norm(h)
            sl = seeds["lora_attn"]
            q, k, v = at.q_proj(a, sl), at.k_proj(a, sl), at.v_proj(a, sl)
            if attn is not None:
                o = attn(torch.cat([q, k, v], -1))
            else:
                q = q.view(B, S, H, hd).transpose(1, 2)
                k = k.view(B, S, H, hd).transpose(1, 2)
                v = v.view(B, S, H, hd).transpose(1, 2)
                o = ref.attention(q, k, v, causal=True, key_padding=key_valid, scale=hd ** -0.5,
                                  dropout_p=cfg.attention_dropout if training else 0.0, seed=seeds["attn"])
                o = o.transpose(1, 2).reshape(B, S, d)
            y = at.out_proj(o, seeds["lora_proj"])
            if training and cfg.dropout > 0:
                y = ref.dropout(y, cfg.dropout, seeds["attn_out"])
            h = h + y
        if parts[1]:
            a2 = self.final_layer_norm(h)
            f = torch.relu(self.fc1(a2, seeds["lora_fc1"]))
            y2 = self.fc2(f, seeds["lora_fc2"])
            if training and cfg.dropout > 0:
                y2 = ref.dropout(y2, cfg.dropout, seeds["mlp_out"])
            h = h + y2
        return h

    def forward_fused(self, h, seeds, training, kv_len=None, attn=None, parts=(True, True)):
        from ..ops import fused as F
        from ..ops.attention import causal_attention
        cfg = self.cfg
        B, S, d = h.shape
        # the MLP's LN backward also runs out_proj's residual-dropout backward + dT (one row pass) when
        # both sub-blocks run here; a half-layer stage boundary between them takes the separate passes
        hand = F.GradHandoff() if training and torch.is_grad_enabled() and parts[0] and parts[1] else None
        if parts[0]:
            at = self.self_attn
            H, hd = at.n_head, at.head_dim
            link = None
            if at.qkv.fusable():
                link = F.ResidualLink()  # residual grad of h enters the LN backward (no separate add)
                qkv = F.ln_linear(h, self.self_attn_layer_norm, at.qkv, seeds["lora_attn"], training, link=link)
            else:  # adapters too wide for one shared K-extension: three projections
                qkv = torch.cat([F.ln_linear(h, self.self_attn_layer_norm, l, seeds["lora_attn"], training)
                                 for l in (at.q_proj, at.k_proj, at.v_proj)], -1)
            if attn is not None:
                o = attn(qkv)
            else:
                o = causal_attention(qkv, B, S, H, hd, scale=hd ** -0.5,
                                     dropout_p=cfg.attention_dropout if training else 0.0, seed=seeds["attn"],
                                     kv_len=kv_len)
            h = F.linear_residual(o, h, at.out_proj, cfg.dropout, seeds["attn_out"], seeds["lora_proj"], training,
                                  link=link, handoff=hand)
        if parts[1]:
            h = F.mlp(h, self.final_layer_norm, self.fc1, self.fc2, act=2, p=cfg.dropout, seed=seeds["mlp_out"],
                      seed_l1=seeds["lora_fc1"], seed_l2=seeds["lora_fc2"], training=training, handoff=hand)
        return h


class OPTLearnedPositionalEmbedding(Embedding):
    OFFSET = 2

    def __init__(self, n_positions, d, dtype=None, device=None):
        super().__init__(n_positions + self.OFFSET, d, dtype=dtype, device=device)


def opt_positions(attention_mask):
    """HF: cumsum(mask)·mask - 1 (pad -> -1; the +2 offset is applied at lookup)."""
    return (torch.cumsum(attention_mask, dim=1) * attention_mask - 1).long()


class OPTForCausalLM(CausalLMBase):
    """HF-compatible OPT LM.  ``forward(input_ids, attention_mask, labels)``.

    ``attention_mask`` is a right-padding key mask (HF tokenizers pad OPT on the
    right); the fused kernels take it as per-row valid lengths."""

    def __init__(self, cfg: OPTConfig, dtype=torch.float32, device=None, layer_range=None, has_embed=True,
                 has_head=True):
        super().__init__()
        self.config = cfg
        self.dtype_ = dtype
        n = cfg.num_hidden_layers
        self.layer_range, self.chunk_ranges, member = normalize_chunks(layer_range, n, halves=True)
        self.has_embed, self.has_head = has_embed, has_head
        d = cfg.hidden_size
        self.model = nn.Module()
        dec = self.model.decoder = nn.Module()
        if has_embed or has_head:
            dec.embed_tokens = Embedding(cfg.vocab_size, d, dtype=dtype, device=device)
        if has_embed:
            dec.embed_positions = OPTLearnedPositionalEmbedding(cfg.max_position_embeddings, d, dtype, device)
        dec.layers = nn.ModuleList(
            [OPTDecoderLayer(cfg, i, dtype, device, chunk_parts(self.chunk_ranges, i)) if member[i] else nn.Identity()
             for i in range(n)])
        if has_head:
            dec.final_layer_norm = LayerNorm(d, cfg.layer_norm_eps, dtype=dtype, device=device)
        self._init_runtime(padded_vocab(cfg.vocab_size))

    def init_weights(self, seed=0):
        init_normal_(self, self.config.init_std, seed=seed)
        return self

    POS_OFFSET = 2

    def tied_embedding(self):
        return self.model.decoder.embed_tokens.weight

    def embedding_tables(self):
        return self.model.decoder.embed_tokens, self.model.decoder.embed_positions

    def final_norm(self):
        return self.model.decoder.final_layer_norm

    def all_blocks(self):
        return [b for b in self.model.decoder.layers if isinstance(b, OPTDecoderLayer)]

    # ---- pieces ----
    def embed_ref(self, input_ids, attention_mask):
        dec = self.model.decoder
        B, S = input_ids.shape
        if attention_mask is None:
            attention_mask = torch.ones(B, S, dtype=torch.long, device=input_ids.device)
        pos = opt_positions(attention_mask) + OPTLearnedPositionalEmbedding.OFFSET
        return dec.embed_tokens(input_ids) + dec.embed_positions(pos)

    def head_ref(self, h, labels, reduction="mean", ignore_index=-100):
        dec = self.model.decoder
        logits = dec.final_layer_norm(h) @ dec.embed_tokens.weight.t()
        if labels is None:
            return None, logits
        return ref_lm_loss(logits, labels, ignore_index, reduction), logits

    def forward(self, input_ids=None, attention_mask=None, labels=None, hidden_states=None, reduction="mean",
                return_logits=True, ignore_index=-100):
        ref_in = input_ids if input_ids is not None else hidden_states
        if self._use_fused(ref_in):
            return self._forward_fused(input_ids, attention_mask, labels, hidden_states, reduction, ignore_index)
        key_valid = attention_mask.bool() if attention_mask is not None else None
        h = self.embed_ref(input_ids, attention_mask) if self.embed_here else hidden_states
        for blk in self.blocks():
            seeds = blk.site_seeds(self.seed, self.micro_step)
            parts = self.block_parts(blk)
            if self.recompute and self.training and torch.is_grad_enabled():
                h = torch.utils.checkpoint.checkpoint(blk.forward_ref, h, seeds, self.training, key_valid, None,
                                                      parts, use_reentrant=False)
            else:
                h = blk.forward_ref(h, seeds, self.training, key_valid, parts=parts)
        if not self.head_here:
            return {"hidden_states": h}
        loss, logits = self.head_ref(h, labels, reduction, ignore_index)
        out = {"loss": loss, "logits": logits if return_logits else None}
        if labels is not None:
            out["ntokens"] = (labels[:, 1:] != ignore_index).sum()
        return out

    def _forward_fused(self, input_ids, attention_mask, labels, hidden_states, reduction, ignore_index):
        from ..ops import fused as F
        from ..ops import kernels as K
        cfg, training = self.config, self.training
        dec = self.model.decoder
        pos = kv_len = None
        if attention_mask is not None:
            if attention_mask.dtype == torch.int64 and attention_mask.is_contiguous():
                pos, kv_len = K.mask_positions(attention_mask)  # one launch for both
            else:
                kv_len = attention_mask.sum(1, dtype=torch.int32)
                pos = opt_positions(attention_mask).contiguous()
        if self.embed_here:
            B, S = input_ids.shape
            h = K.embed(input_ids.contiguous(), dec.embed_tokens.weight, dec.embed_positions.weight, pos=pos,
                        pos_offset=OPTLearnedPositionalEmbedding.OFFSET).view(B, S, -1)
        else:
            h = hidden_states
        for blk in self.blocks():
            seeds = blk.site_seeds(self.seed, self.micro_step)
            parts = self.block_parts(blk)
            if self.recompute and training and torch.is_grad_enabled():
                h = torch.utils.checkpoint.checkpoint(blk.forward_fused, h, seeds, training, kv_len, None, parts,
                                                      use_reentrant=False)
            else:
                h = blk.forward_fused(h, seeds, training, kv_len, parts=parts)
        if not self.head_here:
            return {"hidden_states": h}
        w_nk, w_kn = self.lm_weight_padded(transposed=labels is not None and torch.is_grad_enabled())
        if labels is not None:
            # the causal shift happens inside the head kernels (shift = S); the token count only
            # when a mean is asked for (the trainer normalises by its precomputed global count)
            loss_sum = F.lm_head_xent(h, dec.final_layer_norm, w_nk, labels, cfg.vocab_size, ignore_index,
                                      need_grad=torch.is_grad_enabled(), w_kn=w_kn, shift=labels.shape[-1])
            ntok = (labels[:, 1:] != ignore_index).sum() if reduction == "mean" else None
            loss = loss_sum / ntok.clamp(min=1) if reduction == "mean" else loss_sum
            return {"loss": loss, "logits": None, "ntokens": ntok}
        return {"loss": None, "logits": F.lm_head_logits(h, dec.final_layer_norm, w_nk, cfg.vocab_size)}
