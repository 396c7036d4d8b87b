"""GPT-2 reference path: HF parity, LoRA injection, PEFT save/load, tiny training."""
import json
import os

import pytest
import torch

from mift.models.gpt2 import GPT2Config, GPT2LMHeadModel
from mift import lora as L


def _tiny():
    return GPT2Config(vocab_size=300, n_positions=64, n_embd=64, n_layer=2, n_head=4, n_inner=256)


def _hf_model(cfg):
    transformers = pytest.importorskip("transformers")
    hc = transformers.GPT2Config(vocab_size=cfg.vocab_size, n_positions=cfg.n_positions, n_embd=cfg.n_embd,
                                 n_layer=cfg.n_layer, n_head=cfg.n_head, n_inner=cfg.n_inner,
                                 activation_function="gelu_new", resid_pdrop=0.0, embd_pdrop=0.0,
                                 attn_pdrop=0.0)
    return transformers.GPT2LMHeadModel(hc).eval()


def test_logits_match_hf():
    cfg = _tiny()
    hf = _hf_model(cfg)
    m = GPT2LMHeadModel(cfg)
    sd = {k: v for k, v in hf.state_dict().items() if not k.endswith(".attn.bias") and not k.endswith("masked_bias")}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not [k for k in missing if "lm_head" not in k], missing
    m.eval()
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    with torch.no_grad():
        ref = hf(ids).logits
        out = m(input_ids=ids)["logits"]
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
    lab = ids.clone()
    lab[:, -3:] = -100
    with torch.no_grad():
        l_ref = hf(ids, labels=lab).loss
        l_out = m(input_ids=ids, labels=lab)["loss"]
    torch.testing.assert_close(l_out, l_ref, atol=1e-5, rtol=1e-5)


def test_lora_inject_counts_distilgpt2():
    cfg = GPT2Config.preset("distilgpt2")
    with torch.device("meta"):
        m = GPT2LMHeadModel(cfg)
    names = L.inject(m, L.LoraConfig(r=8, lora_alpha=16, target_modules=["c_attn", "c_proj"]), device="meta")
    n = sum(p.numel() for _, p in L.lora_parameters(m))
    assert n == 405_504
    assert len(names) == 18
    base = sum(p.numel() for n_, p in m.named_parameters() if "lora_" not in n_)
    assert base == 81_912_576


def test_peft_roundtrip(tmp_path):
    cfg = _tiny()
    m = GPT2LMHeadModel(cfg).init_weights(0)
    L.inject(m, L.LoraConfig(r=4, lora_alpha=8, target_modules=["c_attn", "c_proj"]))
    for _, p in L.lora_parameters(m):
        with torch.no_grad():
            p.normal_()
    L.save_pretrained(m, str(tmp_path))
    cfgj = json.load(open(tmp_path / "adapter_config.json"))
    assert cfgj["peft_type"] == "LORA" and cfgj["r"] == 4 and cfgj["fan_in_fan_out"] is True
    from safetensors.torch import load_file
    st = load_file(str(tmp_path / "adapter_model.safetensors"))
    k = "base_model.model.transformer.h.0.attn.c_attn.lora_A.weight"
    assert k in st and tuple(st[k].shape) == (4, 64)
    assert tuple(st["base_model.model.transformer.h.0.attn.c_attn.lora_B.weight"].shape) == (192, 4)
    m2 = GPT2LMHeadModel(cfg).init_weights(0)
    L.inject(m2, L.read_adapter_config(str(tmp_path)))
    L.load_adapter(m2, str(tmp_path))
    for (n1, p1), (n2, p2) in zip(L.lora_parameters(m), L.lora_parameters(m2)):
        assert n1 == n2 and torch.equal(p1, p2)


def test_lora_matches_merged():
    cfg = _tiny()
    m = GPT2LMHeadModel(cfg).init_weights(1).eval()
    L.inject(m, L.LoraConfig(r=4, lora_alpha=8, lora_dropout=0.0, target_modules=["c_attn", "c_proj"]))
    for _, p in L.lora_parameters(m):
        with torch.no_grad():
            p.normal_(0, 0.1)
    ids = torch.randint(0, cfg.vocab_size, (2, 8))
    with torch.no_grad():
        a = m(input_ids=ids)["logits"]
        L.merge_into_base(m)
        b = m(input_ids=ids)["logits"]
    torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-4)
