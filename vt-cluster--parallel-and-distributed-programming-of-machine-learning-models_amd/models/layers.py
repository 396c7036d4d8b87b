"""Building blocks shared by the model families.

Parameter layouts and names are HF-compatible so checkpoints / adapters
interchange with `transformers` + `peft`:
  * ``Linear(conv1d=True)`` stores weight as [in, out] (GPT-2 ``Conv1D``),
    ``conv1d=False`` as [out, in] (``nn.Linear``: OPT, BERT).
  * LoRA matrices hang off the adapted Linear as ``lora_A.weight`` [r, in]
    and ``lora_B.weight`` [out, r] (PEFT's saved key layout).

For the HIP path a frozen Linear also exposes both K-major orientations of
its weight (``w_nk`` = [out,in] for forward, ``w_kn`` = [in,out] for
dgrad).  One of them is the stored parameter itself; the other is built
once and cached (HBM3E is 288 GB: the extra copy buys a single MFMA layout
for every GEMM — see csrc/kernels/gemm.hip).
"""
import math
import zlib

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import reference as ref


class _Mat(nn.Module):
    """A bare ``weight`` holder so state-dict keys read ``lora_A.weight``."""

    def __init__(self, shape, dtype=torch.float32, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(*shape, dtype=dtype, device=device))


class Linear(nn.Module):
    def __init__(self, in_features, out_features, bias=True, conv1d=False, dtype=None, device=None):
        super().__init__()
        self.in_features, self.out_features, self.conv1d = in_features, out_features, conv1d
        shape = (in_features, out_features) if conv1d else (out_features, in_features)
        self.weight = nn.Parameter(torch.empty(*shape, dtype=dtype, device=device))
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=dtype, device=device)) if bias else None
        # LoRA (filled by mift.lora.inject)
        self.lora_r = 0
        self.lora_scaling = 0.0
        self.lora_dropout = 0.0
        self._wcache = {}

    # ---- kernel-layout views of the frozen weight ----
    def _key(self):
        return (self.weight.data_ptr(), self.weight.dtype, self.weight.device)

    def w_nk(self):
        """[out, in] contiguous (forward B operand)."""
        if not self.conv1d:
            return self.weight.detach()
        k = ("nk",) + self._key()
        w = self._wcache.get(k)
        if w is None:
            self._wcache = {kk: v for kk, v in self._wcache.items() if kk[1:] == self._key()}
            w = self.weight.detach().t().contiguous()
            self._wcache[k] = w
        return w

    def w_kn(self):
        """[in, out] contiguous (dgrad B operand)."""
        if self.conv1d:
            return self.weight.detach()
        k = ("kn",) + self._key()
        w = self._wcache.get(k)
        if w is None:
            self._wcache = {kk: v for kk, v in self._wcache.items() if kk[1:] == self._key()}
            w = self.weight.detach().t().contiguous()
            self._wcache[k] = w
        return w

    def drop_cache(self):
        self._wcache = {}

    def has_lora(self):
        return self.lora_r > 0

    # ---- adapter interface of the fused Functions (mift.ops.fused) ----
    def lora_params(self):
        """Trainable adapter tensors, in the order lora_ops().backward() returns grads."""
        return [self.lora_A.weight, self.lora_B.weight] if self.lora_r > 0 else []

    def lora_ops(self, dtype):
        from ..ops.fused import AdapterOps
        return AdapterOps(self, dtype)

    # ---- reference (autograd) path ----
    def forward(self, x, lora_seed=0):
        if self.conv1d:
            y = x @ self.weight
            if self.bias is not None:
                y = y + self.bias
        else:
            y = F.linear(x, self.weight, self.bias)
        if self.lora_r > 0:
            xd = ref.dropout(x, self.lora_dropout, lora_seed) if (self.training and self.lora_dropout > 0) else x
            a = self.lora_A.weight
            b = self.lora_B.weight
            y = y + ((xd.to(a.dtype) @ a.t()) @ b.t()).to(y.dtype) * self.lora_scaling
        return y

    def extra_repr(self):
        s = f"in={self.in_features}, out={self.out_features}, conv1d={self.conv1d}"
        if self.lora_r:
            s += f", lora_r={self.lora_r}, scale={self.lora_scaling}"
        return s


class ConcatLinear:
    """Several Linears that read the same input, run as ONE GEMM.

    OPT keeps q/k/v as separate ``nn.Linear`` (HF / PEFT key names), but on
    the HIP path one [3d, d] GEMM (+ one multi-adapter LoRA K-extension, see
    ``mift.ops.fused.MultiAdapterOps``) writes the fused qkv row that the
    flash-attention kernel reads in place.  Not an nn.Module: it owns no
    parameters, only cached concatenated views of its members' frozen
    weights (rebuilt when any member weight moves)."""

    def __init__(self, lins):
        self.lins = list(lins)
        self.in_features = self.lins[0].in_features
        self.out_features = sum(l.out_features for l in self.lins)
        self._cache = None

    def spans(self):
        n0 = 0
        for l in self.lins:
            yield l, n0, n0 + l.out_features
            n0 += l.out_features

    def _get(self):
        key = tuple((l.weight.data_ptr(), l.weight.dtype) for l in self.lins)
        if self._cache is None or self._cache[0] != key:
            w_nk = torch.cat([l.w_nk() for l in self.lins], 0).contiguous()
            w_kn = torch.cat([l.w_kn() for l in self.lins], 1).contiguous()
            if all(l.bias is None for l in self.lins):
                b = None
            else:
                b = torch.cat([l.bias.detach() if l.bias is not None else
                               torch.zeros(l.out_features, dtype=w_nk.dtype, device=w_nk.device)
                               for l in self.lins])
            self._cache = (key, w_nk, w_kn, b)
        return self._cache

    def w_nk(self):
        return self._get()[1]

    def w_kn(self):
        return self._get()[2]

    @property
    def bias(self):
        return self._get()[3]

    def fusable(self):
        """One shared K-extension fits every member adapter (ranks <= 32 // n)."""
        ad = [l for l in self.lins if l.lora_r > 0]
        if not ad:
            return True
        w = 32 // len(ad)
        return (all(l.lora_r <= w for l in ad) and len({l.lora_dropout for l in ad}) == 1
                and len({getattr(l, "_arena", None) is None for l in ad}) == 1)

    def lora_params(self):
        return [p for l in self.lins for p in l.lora_params()]

    def lora_ops(self, dtype):
        from ..ops.fused import MultiAdapterOps
        return MultiAdapterOps(self, dtype)


class LayerNorm(nn.Module):
    def __init__(self, d, eps=1e-5, dtype=None, device=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(d, dtype=dtype, device=device))
        self.bias = nn.Parameter(torch.zeros(d, dtype=dtype, device=device))

    def forward(self, x):
        return F.layer_norm(x, (x.shape[-1],), self.weight, self.bias, self.eps)


class Embedding(nn.Module):
    def __init__(self, n, d, dtype=None, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(n, d, dtype=dtype, device=device))

    def forward(self, idx):
        return F.embedding(idx, self.weight)


def seed_for(base: int, step: int, site: int) -> int:
    """Deterministic 63-bit dropout seed for (run seed, micro-step, site id)."""
    x = (base * 0x9E3779B97F4A7C15 + step * 0xBF58476D1CE4E5B9 + site * 0x94D049BB133111EB) & ((1 << 64) - 1)
    x ^= x >> 31
    return x & ((1 << 63) - 1)


_GRAPH_SEEDS = [False]


def graph_seeds(on: bool):
    """Switch dropout-site seeds to their step-free form for hipGraph capture (mift.train.graph)."""
    _GRAPH_SEEDS[0] = bool(on)


def dropout_seed(base: int, step: int, site: int) -> int:
    """Seed of a dropout site = ``seed_for(base, step, site)``.  Under hipGraph capture the step is
    read on the device instead (csrc/common.h ``mift_seed``): return the signed 64-bit
    ``base*C1 + site*C3`` and let every replay add its own micro-step."""
    if _GRAPH_SEEDS[0]:
        x = (base * 0x9E3779B97F4A7C15 + site * 0x94D049BB133111EB) & ((1 << 64) - 1)
        return x - (1 << 64) if x >= (1 << 63) else x
    return seed_for(base, step, site)


def name_generator(seed: int, name: str, device=None) -> torch.Generator:
    """RNG keyed by (seed, parameter name): a pipeline stage that builds only some
    layers draws exactly the values the full model would (stage-local init)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "meta":
        return None
    g = torch.Generator(device=dev)
    g.manual_seed(seed_for(seed, 0, zlib.crc32(name.encode())))
    return g


def init_normal_(module: nn.Module, std: float, proj_std: float = None, proj_names=("c_proj",), seed: int = 0):
    """HF-style init: N(0, std) weights, zero biases, unit LayerNorm (per-name RNG streams)."""
    for name, m in module.named_modules():
        if isinstance(m, (Linear, Embedding)):
            s = std
            if isinstance(m, Linear) and proj_std is not None and any(name.endswith(p) for p in proj_names):
                s = proj_std
            with torch.no_grad():
                g = name_generator(seed, name, m.weight.device)
                if g is not None:
                    m.weight.normal_(0.0, s, generator=g)
                if isinstance(m, Linear) and m.bias is not None:
                    m.bias.zero_()
        elif isinstance(m, LayerNorm):
            with torch.no_grad():
                m.weight.fill_(1.0)
                m.bias.zero_()


def causal_attention_ref(q, k, v, dropout_p, seed, scale, key_valid=None):
    """[B,H,S,D] reference attention with counter-hash dropout."""
    return ref.attention(q, k, v, causal=True, key_padding=key_valid, scale=scale, dropout_p=dropout_p, seed=seed)


def padded_vocab(v: int, multiple: int = 128) -> int:
    return int(math.ceil(v / multiple) * multiple)
