"""KV-cache greedy generation == full-recompute greedy and == HF generate (CPU reference path)."""
import pytest
import torch

from mift.infer.generate import generate, generate_nocache
from mift.models.gpt2 import GPT2Config, GPT2LMHeadModel
from mift.models.opt import OPTConfig, OPTForCausalLM


def _gpt2():
    return GPT2LMHeadModel(GPT2Config(vocab_size=300, n_positions=64, n_embd=64, n_layer=2, n_head=4,
                                      n_inner=256)).init_weights(1).eval()


def _opt():
    return OPTForCausalLM(OPTConfig(vocab_size=300, hidden_size=64, num_hidden_layers=2, ffn_dim=256,
                                    num_attention_heads=4, max_position_embeddings=64)).init_weights(2).eval()


@pytest.mark.parametrize("mk", [_gpt2, _opt])
def test_cache_matches_recompute(mk):
    m = mk()
    ids = torch.randint(3, 300, (3, 7))
    a = generate(m, ids, max_new_tokens=9, eos_token_id=-1)
    b = generate_nocache(m, ids, max_new_tokens=9)
    assert torch.equal(a, b)


def test_left_padding_matches_unpadded_rows():
    m = _opt()
    ids = torch.randint(3, 300, (2, 8))
    short = ids[1, 3:]
    batch = ids.clone()
    batch[1, :3] = 1
    mask = torch.ones_like(batch)
    mask[1, :3] = 0
    out = generate(m, batch, attention_mask=mask, max_new_tokens=6, eos_token_id=-1)
    ref0 = generate(m, ids[:1], max_new_tokens=6, eos_token_id=-1)
    ref1 = generate(m, short[None], max_new_tokens=6, eos_token_id=-1)
    assert torch.equal(out[0], ref0[0])
    assert torch.equal(out[1, 3:], ref1[0])


def test_matches_hf_generate_gpt2():
    transformers = pytest.importorskip("transformers")
    m = _gpt2()
    c = m.config
    hf = transformers.GPT2LMHeadModel(transformers.GPT2Config(
        vocab_size=c.vocab_size, n_positions=c.n_positions, n_embd=c.n_embd, n_layer=c.n_layer, n_head=c.n_head,
        n_inner=c.n_inner, activation_function="gelu_new")).eval()
    sd = {k: v for k, v in m.state_dict().items()}
    sd["lm_head.weight"] = sd["transformer.wte.weight"]
    hf.load_state_dict(sd, strict=False)
    ids = torch.randint(3, 300, (2, 5))
    ours = generate(m, ids, max_new_tokens=8, eos_token_id=-1)
    theirs = hf.generate(ids, attention_mask=torch.ones_like(ids), max_new_tokens=8, do_sample=False,
                         pad_token_id=0, eos_token_id=None)
    assert torch.equal(ours, theirs)


def test_eos_then_pad():
    m = _gpt2()
    ids = torch.randint(3, 300, (2, 5))
    free = generate(m, ids, max_new_tokens=6, eos_token_id=-1)
    eos = int(free[0, 5])  # row 0 "finishes" at its first generated token
    out = generate(m, ids, max_new_tokens=6, eos_token_id=eos, pad_token_id=0)
    assert int(out[0, 5]) == eos and (out[0, 6:] == 0).all()
