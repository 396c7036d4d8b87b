"""LoRA: config, injection, flat parameter arena, PEFT-format save/load.

Reference behaviour (`P1/finetune_lora_distilgpt2.py:98-104`,
`P2/finetune_lora_opt_pp.py:104-112`, PEFT [lib]): ``r=8, lora_alpha=16``
(scale alpha/r = 2), ``lora_dropout=0.05``, ``bias="none"``, target modules
matched by name suffix, base weights frozen, ``lora_A`` Kaiming-uniform,
``lora_B`` zeros.  The saved adapter is byte-compatible with PEFT:
``adapter_config.json`` + ``adapter_model.safetensors`` with keys
``base_model.model.<module path>.lora_{A,B}.weight`` (A [r,in], B [out,r]).

MI355X-first addition — the flat arena: all LoRA tensors are views into ONE
fp32 parameter buffer and ONE fp32 gradient buffer (module order), so
  * AdamW (+clip, +unscale/inf-check) is a single multi-tensor-free launch,
  * DDP / ZeRO-1 all-reduce / reduce-scatter one contiguous buffer (or a few
    bucket slices of it), latency-bound on xGMI anyway (0.8-47 MB).
"""
import json
import math
import os
from dataclasses import dataclass, field, asdict
from typing import List, Optional

import torch
import torch.nn as nn

from ..models.layers import Linear, _Mat


@dataclass
class LoraConfig:
    r: int = 8
    lora_alpha: int = 16
    lora_dropout: float = 0.05
    target_modules: List[str] = field(default_factory=lambda: ["c_attn", "c_proj"])
    bias: str = "none"
    task_type: str = "CAUSAL_LM"
    fan_in_fan_out: bool = False
    base_model_name_or_path: Optional[str] = None

    @property
    def scaling(self):
        return self.lora_alpha / self.r

    def to_peft_json(self):
        return {
            "alpha_pattern": {}, "auto_mapping": None,
            "base_model_name_or_path": self.base_model_name_or_path,
            "bias": self.bias, "fan_in_fan_out": self.fan_in_fan_out, "inference_mode": True,
            "init_lora_weights": True, "layers_pattern": None, "layers_to_transform": None,
            "lora_alpha": self.lora_alpha, "lora_dropout": self.lora_dropout, "modules_to_save": None,
            "peft_type": "LORA", "r": self.r, "rank_pattern": {}, "revision": None,
            "target_modules": sorted(self.target_modules), "task_type": self.task_type,
            "use_dora": False, "use_rslora": False,
        }


def _matches(name: str, targets) -> bool:
    return any(name == t or name.endswith("." + t) for t in targets)


def inject(model: nn.Module, cfg: LoraConfig, seed: int = 0, device=None) -> List[str]:
    """Attach LoRA matrices to every Linear whose name matches; freeze the base.

    Returns the adapted module names (in module order)."""
    from ..models.layers import name_generator
    names = []
    for name, m in model.named_modules():
        if isinstance(m, Linear) and _matches(name, cfg.target_modules):
            dev = device or m.weight.device
            m.lora_A = _Mat((cfg.r, m.in_features), torch.float32, dev)
            m.lora_B = _Mat((m.out_features, cfg.r), torch.float32, dev)
            # PEFT init: A ~ kaiming_uniform(a=sqrt(5)) => U(-1/sqrt(in), 1/sqrt(in)); B = 0
            bound = 1.0 / math.sqrt(m.in_features)
            with torch.no_grad():
                # per-module RNG stream: a pipeline stage draws what the full model would
                a = torch.empty(cfg.r, m.in_features).uniform_(-bound, bound,
                                                               generator=name_generator(seed, name + ".lora_A"))
                m.lora_A.weight.copy_(a)
                m.lora_B.weight.zero_()
            m.lora_r = cfg.r
            m.lora_scaling = cfg.scaling
            m.lora_dropout = cfg.lora_dropout
            names.append(name)
    for n, p in model.named_parameters():
        p.requires_grad_(".lora_A." in n or ".lora_B." in n)
    if hasattr(model, "config"):
        cfg.fan_in_fan_out = bool(getattr(model.config, "model_type", "") == "gpt2")
    model.lora_config = cfg
    return names


def lora_parameters(model: nn.Module):
    """(name, param) of every LoRA tensor in module order."""
    return [(n, p) for n, p in model.named_parameters() if ".lora_A." in n or ".lora_B." in n]


class LoraArena:
    """Flat fp32 storage for all LoRA params + grads (see module doc)."""

    def __init__(self, model: nn.Module, device=None, align: int = 64, shards: int = 1, named=None):
        # ``named``: train an explicit parameter list instead (full fine-tuning, e.g. the tiny BERT lab)
        self.named = list(named) if named is not None else lora_parameters(model)
        if not self.named:
            raise ValueError("model has no LoRA parameters (call mift.lora.inject first)")
        device = device or self.named[0][1].device
        self.offsets = []
        off = 0
        for _, p in self.named:
            self.offsets.append(off)
            off += (p.numel() + align - 1) // align * align
        q = align * shards  # ZeRO-1: equal, aligned shards of the flat buffers
        off = (off + q - 1) // q * q
        self.numel = off
        self.n_real = sum(p.numel() for _, p in self.named)
        self.param = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        for (n, p), o in zip(self.named, self.offsets):
            view = self.param[o:o + p.numel()].view_as(p)
            view.copy_(p.detach().to(torch.float32))
            p.data = view
            p.grad = self.grad[o:o + p.numel()].view_as(p)
        self.model = model
        self.version = 0  # bumped whenever the parameters change (optimizer step, load)
        self.grad_ready = None  # fused-backward readiness callback (offsets) set by the DP reducer
        # bind every adapted Linear to its arena slices (fused path writes grads in place)
        off_of = {id(p): o for (_, p), o in zip(self.named, self.offsets)}
        self.modules = []
        for _, m in model.named_modules():
            if isinstance(m, Linear) and m.lora_r > 0 and id(m.lora_A.weight) in off_of:
                m._arena = self
                m._offA = off_of[id(m.lora_A.weight)]
                m._offB = off_of[id(m.lora_B.weight)]
                self.modules.append(m)

    def zero_grad(self):
        self.grad.zero_()

    def bump(self):
        self.version += 1

    def rebind_grads(self):
        """Re-point .grad to the arena (autograd may have replaced it)."""
        if self.grad.is_cuda:
            from ..ops.streams import join
            join()  # side-stream weight-grad kernels (mift.ops.streams) complete before any reader
        for (n, p), o in zip(self.named, self.offsets):
            g = self.grad[o:o + p.numel()].view_as(p)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                if p.grad is not None:
                    g.add_(p.grad)
                p.grad = g

    def state_dict(self):
        return {n: p.detach().clone().cpu() for n, p in self.named}


# ---------------------------------------------------------------------------
# PEFT-format adapter I/O
# ---------------------------------------------------------------------------
PEFT_PREFIX = "base_model.model."


def adapter_state_dict(model: nn.Module):
    return {PEFT_PREFIX + n: p.detach().float().cpu().contiguous() for n, p in lora_parameters(model)}


def save_adapter(save_dir: str, state: dict, cfg: LoraConfig):
    """Write ``adapter_model.safetensors`` + ``adapter_config.json`` (PEFT layout)."""
    from safetensors.torch import save_file
    os.makedirs(save_dir, exist_ok=True)
    save_file({k: v.contiguous() for k, v in state.items()}, os.path.join(save_dir, "adapter_model.safetensors"),
              metadata={"format": "pt"})
    with open(os.path.join(save_dir, "adapter_config.json"), "w") as f:
        json.dump(cfg.to_peft_json(), f, indent=2, sort_keys=True)


def save_pretrained(model: nn.Module, save_dir: str):
    save_adapter(save_dir, adapter_state_dict(model), model.lora_config)


def load_adapter(model: nn.Module, load_dir: str, strict: bool = True):
    """Load a PEFT adapter into an injected model (copies into the arena views)."""
    from safetensors.torch import load_file
    st = load_file(os.path.join(load_dir, "adapter_model.safetensors"))
    own = dict(lora_parameters(model))
    missing = []
    for n, p in own.items():
        k = PEFT_PREFIX + n
        if k not in st:
            missing.append(k)
            continue
        with torch.no_grad():
            p.copy_(st[k].to(p.dtype))
    if strict and missing:
        raise KeyError(f"adapter missing keys: {missing[:5]}")
    return missing


def read_adapter_config(load_dir: str) -> LoraConfig:
    with open(os.path.join(load_dir, "adapter_config.json")) as f:
        d = json.load(f)
    return LoraConfig(r=d["r"], lora_alpha=d["lora_alpha"], lora_dropout=d.get("lora_dropout", 0.0),
                      target_modules=list(d["target_modules"]), bias=d.get("bias", "none"),
                      task_type=d.get("task_type", "CAUSAL_LM"), fan_in_fan_out=d.get("fan_in_fan_out", False),
                      base_model_name_or_path=d.get("base_model_name_or_path"))


def merge_into_base(model: nn.Module):
    """Fold W += s·(B A) into the frozen weights (inference export)."""
    for _, m in model.named_modules():
        if isinstance(m, Linear) and m.lora_r > 0:
            delta = (m.lora_B.weight @ m.lora_A.weight) * m.lora_scaling  # [out, in]
            with torch.no_grad():
                if m.conv1d:
                    m.weight.add_(delta.t().to(m.weight.dtype))
                else:
                    m.weight.add_(delta.to(m.weight.dtype))
                m.lora_B.weight.zero_()
            m.drop_cache()
