"""GPT-2 forward over the fused gfx950 kernels (GPU tensors).

Per block: LN+c_attn(+LoRA) -> causal attention -> c_proj(+LoRA)+dropout+
residual -> LN+c_fc+gelu_new -> c_proj(+LoRA)+dropout+residual; the tied LM
head and the shifted cross-entropy are one Function (mift.ops.fused).
Activations stay [B*S, d] row-major bf16 end to end (no transposes except
the attention head split, which the flash kernel reads in place).
"""
import torch

from ..ops import fused as F
from ..ops import kernels as K
from ..ops.attention import causal_attention


def shift_labels(labels):
    """labels[:, 1:] with an ignore column appended -> aligned with every row."""
    out = torch.full_like(labels, -100)
    out[:, :-1] = labels[:, 1:]
    return out


def block_forward(blk, h, seeds, training):
    cfg = blk.cfg
    B, S, d = h.shape
    H, hd = blk.attn.n_head, blk.attn.head_dim
    qkv = F.ln_linear(h, blk.ln_1, blk.attn.c_attn, seeds["lora_attn"], training)
    o = causal_attention(qkv, B, S, H, hd, scale=hd ** -0.5, dropout_p=cfg.attn_pdrop if training else 0.0,
                         seed=seeds["attn"])
    h = F.linear_residual(o, h, blk.attn.c_proj, cfg.resid_pdrop, seeds["attn_out"], seeds["lora_proj"], training)
    h = F.mlp(h, blk.ln_2, blk.mlp.c_fc, blk.mlp.c_proj, act=1, p=cfg.resid_pdrop, seed=seeds["mlp_out"],
              seed_l1=0, seed_l2=seeds["lora_mlp"], training=training)
    return h


def fused_forward(model, input_ids, attention_mask, labels, hidden_states, reduction, return_logits):
    cfg = model.config
    training = model.training
    if model.has_embed:
        B, S = input_ids.shape
        wte = model.transformer.wte.weight
        h = K.embed(input_ids.contiguous(), wte, model.transformer.wpe.weight,
                    p=cfg.embd_pdrop if training else 0.0, seed=model.embed_seed())
        h = h.view(B, S, -1)
    else:
        h = hidden_states
    for blk in model.blocks():
        seeds = blk.site_seeds(model.seed, model.micro_step)
        if model.recompute and training and torch.is_grad_enabled():
            h = torch.utils.checkpoint.checkpoint(block_forward, blk, h, seeds, training, use_reentrant=False)
        else:
            h = block_forward(blk, h, seeds, training)
    if not model.has_head:
        return {"hidden_states": h}
    w_nk, _ = model.lm_weight_padded()
    if labels is not None:
        sl = shift_labels(labels)
        loss_sum = F.lm_head_xent(h, model.transformer.ln_f, w_nk, sl, cfg.vocab_size, -100,
                                  need_grad=torch.is_grad_enabled())
        ntok = (sl != -100).sum()
        loss = loss_sum / ntok.clamp(min=1) if reduction == "mean" else loss_sum
        return {"loss": loss, "logits": None, "ntokens": ntok}
    logits = F.lm_head_logits(h, model.transformer.ln_f, w_nk, cfg.vocab_size)
    return {"loss": None, "logits": logits}
