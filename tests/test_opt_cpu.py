"""OPT reference path: HF parity (padding-aware positions + key mask), pipeline
stage construction, LoRA injection counts, shared-seed q/k/v LoRA dropout."""
import pytest
import torch

from mift import lora as L
from mift.models.opt import OPTConfig, OPTForCausalLM, opt_positions


def _tiny():
    return OPTConfig(vocab_size=300, hidden_size=64, num_hidden_layers=2, ffn_dim=256, num_attention_heads=4,
                     max_position_embeddings=64)


def _hf(cfg):
    transformers = pytest.importorskip("transformers")
    hc = transformers.OPTConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                                num_hidden_layers=cfg.num_hidden_layers, ffn_dim=cfg.ffn_dim,
                                num_attention_heads=cfg.num_attention_heads,
                                max_position_embeddings=cfg.max_position_embeddings, dropout=0.0,
                                attention_dropout=0.0, word_embed_proj_dim=cfg.hidden_size, pad_token_id=1,
                                do_layer_norm_before=True)
    torch.manual_seed(0)
    return transformers.OPTForCausalLM(hc).eval()


def _ours_from_hf(cfg, hf):
    m = OPTForCausalLM(cfg)
    missing, unexpected = m.load_state_dict(hf.state_dict(), strict=False)
    assert not missing, missing
    assert set(unexpected) <= {"lm_head.weight"}, unexpected
    return m.eval()


def test_logits_match_hf_with_padding():
    cfg = _tiny()
    hf = _hf(cfg)
    m = _ours_from_hf(cfg, hf)
    ids = torch.randint(3, cfg.vocab_size, (2, 16))
    mask = torch.ones(2, 16, dtype=torch.long)
    mask[1, 11:] = 0
    ids[1, 11:] = 1
    with torch.no_grad():
        r = hf(input_ids=ids, attention_mask=mask).logits
        o = m(input_ids=ids, attention_mask=mask)["logits"]
    # padded query rows are don't-care (HF and we both mask their keys only)
    torch.testing.assert_close(o[0], r[0], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(o[1, :11], r[1, :11], atol=1e-4, rtol=1e-4)
    lab = ids.clone()
    lab[mask == 0] = -100
    with torch.no_grad():
        lr = hf(input_ids=ids, attention_mask=mask, labels=lab).loss
        lo = m(input_ids=ids, attention_mask=mask, labels=lab)["loss"]
    torch.testing.assert_close(lo, lr, atol=1e-5, rtol=1e-5)
    # reference OPTHead semantics: ignore_index = pad id on raw input_ids labels
    with torch.no_grad():
        lp = m(input_ids=ids, attention_mask=mask, labels=ids, ignore_index=1)["loss"]
    torch.testing.assert_close(lp, lo, atol=1e-6, rtol=1e-6)


def test_positions_match_hf_rule():
    mask = torch.tensor([[1, 1, 1, 0], [0, 1, 1, 1]])
    assert opt_positions(mask).tolist() == [[0, 1, 2, -1], [-1, 0, 1, 2]]


def test_stage_split_reconstructs_full_model():
    cfg = _tiny()
    full = OPTForCausalLM(cfg).init_weights(3).eval()
    ids = torch.randint(3, cfg.vocab_size, (2, 12))
    with torch.no_grad():
        ref = full(input_ids=ids, labels=ids)["loss"]
    s0 = OPTForCausalLM(cfg, layer_range=(0, 1), has_embed=True, has_head=False).eval()
    s1 = OPTForCausalLM(cfg, layer_range=(1, 2), has_embed=False, has_head=True).eval()
    fsd = full.state_dict()
    for s in (s0, s1):
        sd = s.state_dict()
        assert set(sd) < set(fsd)
        s.load_state_dict({k: fsd[k] for k in sd})
    with torch.no_grad():
        h = s0(input_ids=ids)["hidden_states"]
        loss = s1(hidden_states=h, labels=ids)["loss"]
    torch.testing.assert_close(loss, ref)
    # a middle stage holds no embedding / head weights
    mid = OPTForCausalLM(cfg, layer_range=(1, 2), has_embed=False, has_head=False)
    assert not any("embed" in k or "final_layer_norm.weight" == k.split("decoder.")[-1] for k in mid.state_dict())


def test_half_layer_stages_reconstruct_full_model():
    """Stage boundaries inside a decoder layer (between its attention and MLP sub-blocks): the stages
    hold disjoint weight sets covering the full model exactly and chain to the full model's loss."""
    cfg = _tiny()
    full = OPTForCausalLM(cfg).init_weights(3).eval()
    ids = torch.randint(3, cfg.vocab_size, (2, 12))
    with torch.no_grad():
        ref = full(input_ids=ids, labels=ids)["loss"]
    s0 = OPTForCausalLM(cfg, layer_range=(0, 0.5), has_embed=True, has_head=False).eval()
    s1 = OPTForCausalLM(cfg, layer_range=(0.5, 1.5), has_embed=False, has_head=False).eval()
    s2 = OPTForCausalLM(cfg, layer_range=(1.5, 2), has_embed=False, has_head=True).eval()
    fsd = full.state_dict()
    layer_keys = set()
    for s in (s0, s1, s2):
        sd = s.state_dict()
        assert set(sd) < set(fsd)
        s.load_state_dict({k: fsd[k] for k in sd})
        mine = {k for k in sd if ".layers." in k}
        assert not (mine & layer_keys)  # no sub-block is held twice
        layer_keys |= mine
    assert layer_keys == {k for k in fsd if ".layers." in k}
    assert not any("fc1" in k for k in s0.state_dict()) and not any("q_proj" in k for k in s2.state_dict())
    with torch.no_grad():
        h = s0(input_ids=ids)["hidden_states"]
        h = s1(hidden_states=h)["hidden_states"]
        loss = s2(hidden_states=h, labels=ids)["loss"]
    torch.testing.assert_close(loss, ref)
    from mift.models.gpt2 import GPT2Config, GPT2LMHeadModel
    with pytest.raises(ValueError, match="whole layers"):
        GPT2LMHeadModel(GPT2Config.preset("gpt2-tiny"), layer_range=(0, 0.5))


def test_lora_counts_opt27b():
    cfg = OPTConfig.preset("facebook/opt-2.7b")
    with torch.device("meta"):
        m = OPTForCausalLM(cfg)
    tm = ["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"]
    names = L.inject(m, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=tm), device="meta")
    params = L.lora_parameters(m)
    assert len(names) == 32 * 6 and len(params) == 384   # 384 LoRA tensors
    n = sum(p.numel() for _, p in params)
    assert n == 11_796_480                                 # 4 stages x 2.95 M
    base = sum(p.numel() for k, p in m.named_parameters() if "lora_" not in k)
    assert base == 2_651_596_800                           # facebook/opt-2.7b


def test_lora_shared_seed_ref_path_trains():
    cfg = _tiny()
    m = OPTForCausalLM(cfg).init_weights(1)
    L.inject(m, L.LoraConfig(r=4, lora_alpha=8, target_modules=["q_proj", "k_proj", "v_proj", "out_proj",
                                                                  "fc1", "fc2"]))
    for _, p in L.lora_parameters(m):
        with torch.no_grad():
            p.normal_(0, 0.05)
    m.train()
    ids = torch.randint(3, cfg.vocab_size, (2, 16))
    out = m(input_ids=ids, labels=ids)
    out["loss"].backward()
    g = [p.grad for _, p in L.lora_parameters(m)]
    assert all(x is not None and torch.isfinite(x).all() for x in g)
    assert all(p.grad is None for k, p in m.named_parameters() if "lora_" not in k)
    # same micro_step -> identical dropout masks -> identical loss
    with torch.no_grad():
        l2 = m(input_ids=ids, labels=ids)["loss"]
    torch.testing.assert_close(l2, out["loss"].detach())
