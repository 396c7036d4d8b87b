"""PyTorch reference implementations of every mift kernel.

These run on CPU (the world_size=1 gloo plumbing configuration and the CPU
test-suite) and are the numerics oracle for the HIP kernels (tests compare
kernel output against these evaluated in fp32).

Dropout uses the same counter hash as ``csrc/common.h::mift_hash`` so a
mask drawn on the GPU can be reproduced bit-for-bit on the CPU.
"""
import math

import torch
import torch.nn.functional as F

_M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 on uint32 values held in int64 tensors (matches csrc/common.h)."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


def mift_hash_pair(seed: int, pair: torch.Tensor) -> torch.Tensor:
    seed &= (1 << 64) - 1
    lo = pair & _M32
    hi = (pair >> 32) & _M32
    s_lo, s_hi = seed & _M32, (seed >> 32) & _M32
    return _mix32(((lo * 0x9E3779B9) & _M32) ^ _mix32(hi ^ s_hi) ^ s_lo)


def mift_bits16(seed: int, idx: torch.Tensor) -> torch.Tensor:
    idx = idx.to(torch.int64)
    h = mift_hash_pair(seed, idx >> 1)
    return (h >> ((idx & 1) * 16)) & 0xFFFF


def thr16(p: float) -> int:
    return 0 if p <= 0 else min(int(p * 65536.0 + 0.5), 65536)


def inv_keep(p: float) -> float:
    t = thr16(p)
    return 1.0 if t == 0 else (0.0 if t >= 65536 else 65536.0 / (65536.0 - t))


def keep_mask(seed: int, shape, p: float, device=None) -> torch.Tensor:
    """Boolean keep-mask for a row-major tensor of `shape` (idx = linear index)."""
    n = 1
    for s in shape:
        n *= int(s)
    idx = torch.arange(n, dtype=torch.int64, device=device)
    return (mift_bits16(seed, idx) >= thr16(p)).view(*shape)


def dropout(x: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    if p <= 0.0:
        return x
    m = keep_mask(seed, x.shape, p, x.device)
    return torch.where(m, x * inv_keep(p), torch.zeros((), dtype=x.dtype, device=x.device))


def gelu_new(x: torch.Tensor) -> torch.Tensor:
    """GPT-2 gelu_new (tanh approximation), HF ``NewGELUActivation``."""
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


ACT_NONE, ACT_GELU_TANH, ACT_RELU, ACT_GELU_ERF = 0, 1, 2, 3
ACT_GELU_TANH_BWD, ACT_RELU_BWD, ACT_GELU_ERF_BWD = 4, 5, 6


def _act(act, z, aux):
    if act == ACT_NONE:
        return z
    if act == ACT_GELU_TANH:
        return gelu_new(z)
    if act == ACT_RELU:
        return torch.relu(z)
    if act == ACT_GELU_ERF:
        return F.gelu(z)
    if act == ACT_GELU_TANH_BWD:
        a = aux.float().requires_grad_(True)
        with torch.enable_grad():
            g, = torch.autograd.grad(gelu_new(a).sum(), a)
        return z * g
    if act == ACT_RELU_BWD:
        return torch.where(aux > 0, z, torch.zeros_like(z))
    if act == ACT_GELU_ERF_BWD:
        a = aux.float().requires_grad_(True)
        with torch.enable_grad():
            g, = torch.autograd.grad(F.gelu(a).sum(), a)
        return z * g
    raise ValueError(act)


def gemm_nt(a, b, bias=None, a2=None, b2=None, act=ACT_NONE, aux=None, residual=None,
            dropout_p=0.0, seed=0, want_preact=False, alpha=1.0, out_dtype=None):
    """Semantics of ``_C.gemm_nt`` evaluated in fp32 (rounding points match:
    z is rounded to the output dtype before the elementwise tail)."""
    odt = out_dtype or a.dtype
    z = a.float() @ b.float().t()
    if a2 is not None:
        z = z + a2.float() @ b2.float().t()
    z = z * alpha
    if bias is not None:
        z = z + bias.float()
    z = z.to(odt).float()
    pre = z.to(odt) if want_preact else None
    y = _act(act, z, aux.float() if aux is not None else None)
    if dropout_p > 0:
        y = dropout(y, dropout_p, seed)
    if residual is not None:
        y = y + residual.float()
    return y.to(odt), pre


def layer_norm(x, w, b, eps):
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def attention(q, k, v, causal=True, key_padding=None, scale=None, dropout_p=0.0, seed=0):
    """q,k,v: [B, H, S, D].  key_padding: [B, S] bool (True = valid)."""
    B, H, S, D = q.shape
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    Sk = k.shape[2]
    mask = torch.zeros(B, 1, S, Sk, dtype=torch.bool, device=q.device)
    if causal:
        cm = torch.ones(S, Sk, dtype=torch.bool, device=q.device).tril(Sk - S)
        mask = mask | ~cm
    if key_padding is not None:
        mask = mask | ~key_padding[:, None, None, :].bool()
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    if dropout_p > 0:
        p = dropout(p, dropout_p, seed)
    return (p @ v.float()).to(q.dtype)


def cross_entropy(logits, labels, ignore_index=-100, reduction="mean"):
    return F.cross_entropy(logits.float(), labels, ignore_index=ignore_index, reduction=reduction)
