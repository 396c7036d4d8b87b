"""GPT-2 forward over the fused gfx950 kernels (GPU tensors).

Per block (``GPT2Block.forward_fused``): LN+c_attn(+LoRA) -> causal
attention -> c_proj(+LoRA)+dropout+residual -> LN+c_fc+gelu_new ->
c_proj(+LoRA)+dropout+residual; the tied LM head and the shifted
cross-entropy are one Function (mift.ops.fused).  Activations stay
[B*S, d] row-major 16-bit end to end (no transposes: the flash kernel reads
the fused qkv row in place).
"""
import torch

from ..ops import fused as F
from ..ops import kernels as K
from .base import shift_labels  # noqa: F401  (re-export, used by callers)


def block_forward(blk, h, seeds, training, kv_len=None):
    return blk.forward_fused(h, seeds, training, kv_len)


def fused_forward(model, input_ids, attention_mask, labels, hidden_states, reduction, return_logits):
    cfg = model.config
    training = model.training
    if model.embed_here:
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
            h = torch.utils.checkpoint.checkpoint(blk.forward_fused, h, seeds, training, use_reentrant=False)
        else:
            h = blk.forward_fused(h, seeds, training)
    if not model.head_here:
        return {"hidden_states": h}
    w_nk, w_kn = model.lm_weight_padded(transposed=labels is not None and torch.is_grad_enabled())
    if labels is not None:
        # causal shift inside the head kernels (shift = S); token count only for a mean
        loss_sum = F.lm_head_xent(h, model.transformer.ln_f, w_nk, labels, cfg.vocab_size, -100,
                                  need_grad=torch.is_grad_enabled(), w_kn=w_kn, shift=labels.shape[-1])
        ntok = (labels[:, 1:] != -100).sum() if reduction == "mean" else None
        loss = loss_sum / ntok.clamp(min=1) if reduction == "mean" else loss_sum
        return {"loss": loss, "logits": None, "ntokens": ntok}
    logits = F.lm_head_logits(h, model.transformer.ln_f, w_nk, cfg.vocab_size)
    return {"loss": None, "logits": logits}
