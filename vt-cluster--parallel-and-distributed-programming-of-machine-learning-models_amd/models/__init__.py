"""Model families: GPT-2 (distilgpt2), OPT (2.7B / 6.7B / small), BERT (tiny lab,
RoBERTa/DistilBERT-style encoders), T5 (RAG generator).

``build_causal_lm(name, ...)`` maps a reference model id (``distilgpt2``,
``facebook/opt-2.7b`` ...) to our implementation with HF-compatible
parameter names; weights are random-initialised (no network) unless a local
HF checkpoint directory is given.
"""
import json
import os

import torch


def build_causal_lm(name: str, dtype=torch.float32, device=None, seed: int = 0, weights: str = None,
                    layer_range=None, has_embed=True, has_head=True, init=True):
    n = name.lower()
    if "opt" in n:
        from .opt import OPTConfig, OPTForCausalLM
        cfg = OPTConfig.preset(name)
        m = OPTForCausalLM(cfg, dtype=dtype, device=device, layer_range=layer_range, has_embed=has_embed,
                           has_head=has_head)
    else:
        from .gpt2 import GPT2Config, GPT2LMHeadModel
        cfg = GPT2Config.preset(name)
        m = GPT2LMHeadModel(cfg, dtype=dtype, device=device, layer_range=layer_range, has_embed=has_embed,
                            has_head=has_head)
    if weights:
        load_hf_weights(m, weights)
    elif init:
        m.init_weights(seed)
    m.name_or_path = name
    return m


def load_hf_weights(model, path: str, strict: bool = False):
    """Load a local HF checkpoint dir (safetensors or pytorch_model.bin, weights_only)."""
    sd = {}
    st = [f for f in os.listdir(path) if f.endswith(".safetensors")]
    if st:
        from safetensors.torch import load_file
        for f in st:
            sd.update(load_file(os.path.join(path, f)))
    else:
        for f in os.listdir(path):
            if f.endswith(".bin"):
                sd.update(torch.load(os.path.join(path, f), map_location="cpu", weights_only=True))
    own = model.state_dict()
    mapped = {}
    for k, v in sd.items():
        kk = k
        if kk not in own and ("model." + kk) in own:
            kk = "model." + kk
        if kk in own and own[kk].shape == v.shape:
            mapped[kk] = v.to(own[kk].dtype)
    model.load_state_dict(mapped, strict=False)
    return sorted(set(own) - set(mapped))


def save_hf_config(model, d):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(model.config.to_hf_dict(), f, indent=2)


def save_hf_model(model, d):
    """HF-layout checkpoint dir: ``model.safetensors`` (all weights) + ``config.json``."""
    from safetensors.torch import save_file
    os.makedirs(d, exist_ok=True)
    save_file({k: v.detach().contiguous().cpu() for k, v in model.state_dict().items()},
              os.path.join(d, "model.safetensors"), metadata={"format": "pt"})
    save_hf_config(model, d)
