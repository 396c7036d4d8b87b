"""K3 causal self-attention entry point.

``causal_attention(qkv, B, S, H, hd, ...)`` takes the fused projection output
[B, S, 3*H*hd] (q | k | v, heads interleaved as HF GPT-2 / OPT split them)
and returns [B, S, H*hd].  GPU tensors run the gfx950 flash-attention
kernels (csrc/kernels/attention.hip) when available for the head dim;
otherwise (CPU) the reference path.
"""
import os

import torch
import torch.nn.functional as Fnn

from . import reference as ref
from .dispatch import use_kernels, C


def _split(qkv, B, S, H, hd):
    x = qkv.view(B, S, 3, H, hd)
    return x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)


class _FlashAttn(torch.autograd.Function):
    """With dropout the forward also returns its keep-bit record (whole-sequence kernels, see
    KEEP BITS in csrc/kernels/attention.hip) and the backward reads it instead of re-hashing
    (``MIFT_ATTN_BITS=0``: re-hash, for A/B measurements; read per call, i.e. at graph capture)."""

    @staticmethod
    def forward(ctx, qkv, B, S, H, hd, scale, p, seed, kv_len):
        qkv = qkv.contiguous()
        if p > 0 and os.environ.get("MIFT_ATTN_BITS", "1") != "0":
            o, lse, bits = C().attn_fwd_bits(qkv, B, S, H, hd, float(scale), float(p), int(seed), kv_len)
        else:
            (o, lse), bits = C().attn_fwd(qkv, B, S, H, hd, float(scale), float(p), int(seed), kv_len), None
        ctx.save_for_backward(qkv, o, lse, kv_len if kv_len is not None else torch.empty(0),
                              bits if bits is not None else torch.empty(0))
        ctx.meta = (B, S, H, hd, scale, p, seed, kv_len is not None)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, kv_len, bits = ctx.saved_tensors
        B, S, H, hd, scale, p, seed, has_len = ctx.meta
        dqkv = C().attn_bwd_bits(do.contiguous(), qkv, o, lse, B, S, H, hd, float(scale), float(p), int(seed),
                                 kv_len if has_len else None, bits if bits.numel() else None)
        return dqkv, None, None, None, None, None, None, None, None


def flash_supported(hd):
    try:
        return hasattr(C(), "attn_fwd") and hd in (32, 64, 80, 128)
    except Exception:
        return False


def causal_attention(qkv, B, S, H, hd, scale=None, dropout_p=0.0, seed=0, kv_len=None):
    scale = scale if scale is not None else hd ** -0.5
    if use_kernels(qkv) and flash_supported(hd):
        o = _FlashAttn.apply(qkv.reshape(B * S, 3 * H * hd), B, S, H, hd, scale, dropout_p, seed, kv_len)
        return o.view(B, S, H * hd)
    q, k, v = _split(qkv, B, S, H, hd)
    if qkv.is_cuda:
        # GPU without the flash kernel for this head dim: torch SDPA (its own RNG for dropout)
        o = Fnn.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=True, scale=scale)
    else:
        valid = None
        if kv_len is not None:
            valid = torch.arange(S, device=qkv.device)[None, :] < kv_len[:, None]
        o = ref.attention(q, k, v, causal=True, key_padding=valid, scale=scale, dropout_p=dropout_p, seed=seed)
    return o.transpose(1, 2).reshape(B, S, H * hd)
