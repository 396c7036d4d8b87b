"""K12 decode attention kernel + fused KV-cache generation on the GPU."""
import pytest
import torch

from mift.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("hd", [64, 80, 128])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_decode_attn_kernel(hd, dt):
    from mift.ops import kernels as K
    torch.manual_seed(0)
    B, H, Tmax, t = 3, 4, 300, 257
    kc = torch.randn(B, H, Tmax, hd, device="cuda").to(dt)
    vc = torch.randn(B, H, Tmax, hd, device="cuda").to(dt)
    qkv = torch.randn(B, 3 * H * hd, device="cuda").to(dt)
    start = torch.tensor([0, 5, 100], device="cuda", dtype=torch.int32)
    kc0, vc0 = kc.clone(), vc.clone()
    o = K.decode_attn(qkv, kc, vc, t, hd ** -0.5, start)
    d = H * hd
    kref, vref = kc0.clone(), vc0.clone()
    kref[:, :, t] = qkv[:, d:2 * d].view(B, H, hd)
    vref[:, :, t] = qkv[:, 2 * d:].view(B, H, hd)
    assert torch.equal(kc[:, :, t], kref[:, :, t]) and torch.equal(vc[:, :, t], vref[:, :, t])
    q = qkv[:, :d].view(B, H, 1, hd)
    valid = torch.arange(t + 1, device="cuda")[None, :] >= start[:, None].long()
    oref = ref.attention(q.float(), kref[:, :, :t + 1].float(), vref[:, :, :t + 1].float(), causal=False,
                         key_padding=valid, scale=hd ** -0.5)
    torch.testing.assert_close(o.float(), oref.transpose(1, 2).reshape(B, d), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("name", ["gpt2", "opt"])
def test_fused_generate_matches_recompute(name):
    from mift.infer.generate import generate, generate_nocache
    from mift.models.gpt2 import GPT2Config, GPT2LMHeadModel
    from mift.models.opt import OPTConfig, OPTForCausalLM
    if name == "gpt2":
        m = GPT2LMHeadModel(GPT2Config(vocab_size=1000, n_positions=128, n_embd=128, n_layer=2, n_head=2,
                                       n_inner=512), dtype=torch.bfloat16, device="cuda").init_weights(1)
    else:
        m = OPTForCausalLM(OPTConfig(vocab_size=1000, hidden_size=320, num_hidden_layers=2, ffn_dim=1280,
                                     num_attention_heads=4, max_position_embeddings=128), dtype=torch.float16,
                           device="cuda").init_weights(2)
    m.eval()
    torch.manual_seed(3)
    ids = torch.randint(3, 1000, (4, 24), device="cuda")
    a = generate(m, ids, max_new_tokens=10, eos_token_id=-1)
    b = generate_nocache(m, ids, max_new_tokens=10)
    # 16-bit: a near-tie argmax may flip between the cached and recomputed paths; demand >= 90 % agreement
    agree = (a[:, 24:] == b[:, 24:]).float().mean().item()
    assert agree >= 0.9, (agree, a[:, 24:], b[:, 24:])
    # left-padded batch: padded row == its unpadded run
    batch = ids.clone()
    batch[1, :6] = 1
    mask = torch.ones_like(batch)
    mask[1, :6] = 0
    out = generate(m, batch, attention_mask=mask, max_new_tokens=6, eos_token_id=-1)
    solo = generate(m, ids[1:2, 6:], max_new_tokens=6, eos_token_id=-1)
    assert (out[1, 24:] == solo[0, 18:]).float().mean().item() >= 0.8


@pytest.mark.parametrize("hd", [64, 80])
def test_decode_attn_prompt_gap(hd):
    """Right-aligned prompts (generate.py): keys in [plen[b], gend) are masked; the rest exact."""
    from mift.ops import kernels as K
    torch.manual_seed(1)
    B, H, Tmax, t, gend = 3, 2, 64, 40, 30
    dt = torch.bfloat16
    kc = torch.randn(B, H, Tmax, hd, device="cuda").to(dt)
    vc = torch.randn(B, H, Tmax, hd, device="cuda").to(dt)
    qkv = torch.randn(B, 3 * H * hd, device="cuda").to(dt)
    plen = torch.tensor([30, 7, 1], device="cuda", dtype=torch.int32)
    kc0, vc0 = kc.clone(), vc.clone()
    o = K.decode_attn(qkv, kc, vc, t, hd ** -0.5, plen=plen, gend=gend)
    d = H * hd
    kref, vref = kc0.clone(), vc0.clone()
    kref[:, :, t] = qkv[:, d:2 * d].view(B, H, hd)
    vref[:, :, t] = qkv[:, 2 * d:].view(B, H, hd)
    j = torch.arange(t + 1, device="cuda")[None, :]
    valid = (j < plen[:, None].long()) | (j >= gend)
    q = qkv[:, :d].view(B, H, 1, hd)
    oref = ref.attention(q.float(), kref[:, :, :t + 1].float(), vref[:, :, :t + 1].float(), causal=False,
                         key_padding=valid, scale=hd ** -0.5)
    torch.testing.assert_close(o.float(), oref.transpose(1, 2).reshape(B, d), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("name", ["gpt2", "opt"])
def test_padded_distinct_prompts_match_solo_nocache(name):
    """The probe's padded path: 16 DIFFERENT left-padded prompts generated as one batch (flash prefill
    over right-aligned prompts, gap-masked decode, gemm_nt logits) give each row the tokens of its
    own unpadded prompt run without a cache (full recompute per token)."""
    from mift.apps.gen_probe import distinct_prompts
    from mift.infer.generate import generate, generate_nocache
    from mift.models.gpt2 import GPT2Config, GPT2LMHeadModel
    from mift.models.opt import OPTConfig, OPTForCausalLM
    if name == "gpt2":
        m = GPT2LMHeadModel(GPT2Config(vocab_size=1000, n_positions=128, n_embd=128, n_layer=2, n_head=2,
                                       n_inner=512), dtype=torch.bfloat16, device="cuda").init_weights(1)
    else:
        m = OPTForCausalLM(OPTConfig(vocab_size=1000, hidden_size=320, num_hidden_layers=2, ffn_dim=1280,
                                     num_attention_heads=4, max_position_embeddings=128), dtype=torch.float16,
                           device="cuda").init_weights(2)
    m.eval()
    ids, mask = distinct_prompts(16, 1000, 1, "cuda")
    S0 = ids.shape[1]
    out = generate(m, ids, attention_mask=mask, max_new_tokens=8, eos_token_id=-1)
    assert out.shape == (16, S0 + 8) and torch.equal(out[:, :S0], ids)
    agree, total = 0, 0
    for b in range(16):
        L = int(mask[b].sum())
        solo = generate_nocache(m, ids[b:b + 1, S0 - L:], max_new_tokens=8)
        agree += int((solo[0, L:] == out[b, S0:]).sum())
        total += 8
    print(f"{name}: padded-batch vs solo no-cache token agreement {agree}/{total}")
    assert agree >= 0.95 * total, (agree, total)


def test_decode_attn_device_position_matches_host():
    """decode_attn with the position in an int32 device tensor (graph-replayed decode) == host int."""
    from mift.ops import kernels as K
    torch.manual_seed(2)
    B, H, hd, Tmax, t = 2, 3, 64, 96, 70
    dt = torch.bfloat16
    kc = torch.randn(B, H, Tmax, hd, device="cuda").to(dt)
    vc = torch.randn(B, H, Tmax, hd, device="cuda").to(dt)
    qkv = torch.randn(B, 3 * H * hd, device="cuda").to(dt)
    plen = torch.tensor([9, 31], device="cuda", dtype=torch.int32)
    k1, v1, k2, v2 = kc.clone(), vc.clone(), kc.clone(), vc.clone()
    o1 = K.decode_attn(qkv, k1, v1, t, hd ** -0.5, plen=plen, gend=40)
    o2 = K.decode_attn(qkv, k2, v2, torch.tensor([t], dtype=torch.int32, device="cuda"), hd ** -0.5, plen=plen,
                       gend=40)
    assert torch.equal(o1, o2) and torch.equal(k1, k2) and torch.equal(v1, v2)


@pytest.mark.parametrize("name", ["gpt2", "opt"])
def test_graphed_decode_matches_eager(name, monkeypatch):
    """A whole generate() call replayed from one hipGraph (prefill + device-side position / flags / output
    column) gives the eager loop's tokens exactly, for left-padded batches, for new inputs of a cached
    shape and with HF's stop-when-all-finished rule."""
    from mift.apps.gen_probe import distinct_prompts
    from mift.infer import generate as G
    from mift.models.gpt2 import GPT2Config, GPT2LMHeadModel
    from mift.models.opt import OPTConfig, OPTForCausalLM
    if name == "gpt2":
        m = GPT2LMHeadModel(GPT2Config(vocab_size=1000, n_positions=128, n_embd=128, n_layer=2, n_head=2,
                                       n_inner=512), dtype=torch.bfloat16, device="cuda").init_weights(1)
    else:
        m = OPTForCausalLM(OPTConfig(vocab_size=1000, hidden_size=320, num_hidden_layers=2, ffn_dim=1280,
                                     num_attention_heads=4, max_position_embeddings=128), dtype=torch.float16,
                           device="cuda").init_weights(2)
    m.eval()
    ids, mask = distinct_prompts(16, 1000, 1, "cuda")

    def both(**kw):
        monkeypatch.setenv("MIFT_GEN_GRAPH", "0")
        e = G.generate(m, ids, attention_mask=mask, **kw)
        monkeypatch.setenv("MIFT_GEN_GRAPH", "1")
        g1 = G.generate(m, ids, attention_mask=mask, **kw)  # captures
        g2 = G.generate(m, ids, attention_mask=mask, **kw)  # replays the cached graph
        return e, g1, g2

    e, g1, g2 = both(max_new_tokens=12, eos_token_id=-1)
    assert e.shape == (16, ids.shape[1] + 12) and torch.equal(e, g1) and torch.equal(e, g2)
    # the cached whole-call graph (prefill included) on NEW inputs of the same shape: rows reordered,
    # so every row's prompt length and tokens change
    ids_f, mask_f = ids.flip(0).contiguous(), mask.flip(0).contiguous()
    monkeypatch.setenv("MIFT_GEN_GRAPH", "0")
    e_f = G.generate(m, ids_f, attention_mask=mask_f, max_new_tokens=12, eos_token_id=-1)
    monkeypatch.setenv("MIFT_GEN_GRAPH", "1")
    g_f = G.generate(m, ids_f, attention_mask=mask_f, max_new_tokens=12, eos_token_id=-1)
    assert torch.equal(e_f, g_f) and torch.equal(e_f, e.flip(0))
    # a budget above the unroll limit: the prefill graph, then one step graph replayed per token
    monkeypatch.setenv("MIFT_GEN_UNROLL", "4")
    G._GRAPHS.clear()
    s1 = G.generate(m, ids, attention_mask=mask, max_new_tokens=12, eos_token_id=-1)
    s2 = G.generate(m, ids, attention_mask=mask, max_new_tokens=12, eos_token_id=-1)
    assert torch.equal(e, s1) and torch.equal(e, s2)
    monkeypatch.delenv("MIFT_GEN_UNROLL")
    G._GRAPHS.clear()
    # early stop: identical prompts -> identical rows; EOS := the 4th generated token
    same = ids[:1].expand(4, -1).contiguous()
    msk = mask[:1].expand(4, -1).contiguous()
    monkeypatch.setenv("MIFT_GEN_GRAPH", "0")
    ref_out = G.generate(m, same, attention_mask=msk, max_new_tokens=12, eos_token_id=-1)
    eos = int(ref_out[0, same.shape[1] + 3])
    e = G.generate(m, same, attention_mask=msk, max_new_tokens=12, eos_token_id=eos)
    monkeypatch.setenv("MIFT_GEN_GRAPH", "1")
    g = G.generate(m, same, attention_mask=msk, max_new_tokens=12, eos_token_id=eos)
    assert e.shape[1] <= same.shape[1] + 4 and torch.equal(e, g), (e.shape, g.shape)


@pytest.mark.parametrize("hd,dt", [(64, torch.bfloat16), (80, torch.float16), (128, torch.bfloat16)])
def test_kv_store_matches_strided_copies(hd, dt):
    """kv_store (prefill, one launch) writes exactly the rows the two strided cache copies wrote."""
    from mift.ops import kernels as K
    torch.manual_seed(2)
    B, H, S, Tmax = 3, 5, 37, 50
    d = H * hd
    qkv = torch.randn(B * S, 3 * d, device="cuda").to(dt)
    kc = torch.randn(B, H, Tmax, hd, device="cuda").to(dt)
    vc = torch.randn(B, H, Tmax, hd, device="cuda").to(dt)
    kr, vr = kc.clone(), vc.clone()
    q3 = qkv.view(B, S, 3 * d)
    kr[:, :, :S].copy_(q3[..., d:2 * d].view(B, S, H, hd).transpose(1, 2))
    vr[:, :, :S].copy_(q3[..., 2 * d:].view(B, S, H, hd).transpose(1, 2))
    K.kv_store(qkv, kc, vc, S)
    assert torch.equal(kc, kr) and torch.equal(vc, vr)


def test_graphed_generate_follows_adapter_updates(monkeypatch):
    """the cached whole-call decode graph must not replay stale LoRA operands.  OPT with
    adapters on q / v (one multi-adapter K-extension) and fc1: generate (capture + replay), change the
    adapters in place through the arena as an optimizer step does (version bump), generate again —
    every graphed call equals the eager path (MIFT_GEN_GRAPH=0) on the weights of that moment."""
    from mift import lora as L
    from mift.apps.gen_probe import distinct_prompts
    from mift.infer import generate as G
    from mift.models.opt import OPTConfig, OPTForCausalLM
    m = OPTForCausalLM(OPTConfig(vocab_size=1000, hidden_size=320, num_hidden_layers=2, ffn_dim=1280,
                                 num_attention_heads=4, max_position_embeddings=128), dtype=torch.float16,
                       device="cuda").init_weights(3)
    L.inject(m, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=["q_proj", "v_proj", "fc1"]))
    arena = L.LoraArena(m)
    g = torch.Generator(device="cuda").manual_seed(0)
    with torch.no_grad():
        arena.param.copy_(torch.randn(arena.param.shape, device="cuda", generator=g) * 0.2)
    arena.bump()
    m.eval()
    ids, mask = distinct_prompts(16, 1000, 1, "cuda")

    def both():
        monkeypatch.setenv("MIFT_GEN_GRAPH", "0")
        e = G.generate(m, ids, attention_mask=mask, max_new_tokens=10, eos_token_id=-1)
        monkeypatch.setenv("MIFT_GEN_GRAPH", "1")
        g1 = G.generate(m, ids, attention_mask=mask, max_new_tokens=10, eos_token_id=-1)
        g2 = G.generate(m, ids, attention_mask=mask, max_new_tokens=10, eos_token_id=-1)
        return e, g1, g2

    e0, a0, b0 = both()
    assert torch.equal(e0, a0) and torch.equal(e0, b0)
    with torch.no_grad():  # an "optimizer step": new adapter values in place, version bumped
        arena.param.add_(torch.randn(arena.param.shape, device="cuda", generator=g) * 0.5)
    arena.bump()
    e1, a1, b1 = both()
    assert torch.equal(e1, a1) and torch.equal(e1, b1)
    assert not torch.equal(e0, e1)  # the adapters matter: the update changed the tokens
