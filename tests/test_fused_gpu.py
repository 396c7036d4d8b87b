"""Fused HIP GPT-2 path vs the fp32 reference path (same weights, dropout off)."""
import copy

import pytest
import torch

import mift
from mift import lora as L
from mift.models.gpt2 import GPT2Config, GPT2LMHeadModel

pytestmark = pytest.mark.gpu


def _models(dropout=0.0):
    cfg = GPT2Config(vocab_size=1000, n_positions=128, n_embd=128, n_layer=2, n_head=2, n_inner=512,
                     embd_pdrop=dropout, attn_pdrop=dropout, resid_pdrop=dropout)
    ref = GPT2LMHeadModel(cfg, dtype=torch.float32, device="cuda").init_weights(3)
    L.inject(ref, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=dropout, target_modules=["c_attn", "c_proj"]))
    for _, p in L.lora_parameters(ref):
        with torch.no_grad():
            p.normal_(0, 0.05)
    fused = copy.deepcopy(ref)
    for n, p in fused.named_parameters():
        if "lora_" not in n:
            p.data = p.data.to(torch.bfloat16)
    ref.fused = False
    return cfg, ref, fused


def test_fused_matches_reference_loss_and_grads():
    assert mift.kernels_available(), mift._ext.error()
    cfg, ref, fused = _models(0.0)
    torch.manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (4, 64), device="cuda")
    lab = ids.clone()
    lab[:, -5:] = -100
    ref.train()
    fused.train()
    lr = ref(input_ids=ids, labels=lab, reduction="sum")["loss"]
    lr.backward()
    lf = fused(input_ids=ids, labels=lab, reduction="sum")["loss"]
    lf.backward()
    torch.testing.assert_close(lf.float(), lr.float(), rtol=2e-2, atol=1e-1)
    for (n1, p1), (n2, p2) in zip(L.lora_parameters(ref), L.lora_parameters(fused)):
        g1, g2 = p1.grad.float(), p2.grad.float()
        rel = (g1 - g2).norm() / (g1.norm() + 1e-6)
        assert rel < 5e-2, f"{n1}: rel err {rel:.3e}"


def test_fused_dropout_runs_and_is_deterministic():
    cfg, ref, fused = _models(0.1)
    ids = torch.randint(0, cfg.vocab_size, (2, 64), device="cuda")
    fused.train()
    fused.micro_step = 7
    a = fused(input_ids=ids, labels=ids, reduction="sum")["loss"].item()
    b = fused(input_ids=ids, labels=ids, reduction="sum")["loss"].item()
    assert abs(a - b) < 1e-3 * abs(a)  # same micro_step -> same masks (flash path) or close (sdpa)


def test_arena_pack_path_matches_dense_path():
    """Trainer fast path (packed operands + grads written into the arena) == per-module path."""
    from mift.lora import LoraArena
    from mift.lora.pack import attach
    cfg, ref, fused = _models(0.0)
    fused2 = copy.deepcopy(fused)
    ids = torch.randint(0, cfg.vocab_size, (4, 64), device="cuda")
    fused.train()
    fused2.train()
    fused(input_ids=ids, labels=ids, reduction="sum")["loss"].backward()
    arena = LoraArena(fused2)
    attach(fused2, arena, torch.bfloat16)
    fused2(input_ids=ids, labels=ids, reduction="sum")["loss"].backward()
    for (n1, p1), (n2, p2) in zip(L.lora_parameters(fused), L.lora_parameters(fused2)):
        g1, g2 = p1.grad.float(), p2.grad.float()
        rel = (g1 - g2).norm() / (g1.norm() + 1e-6)
        assert rel < 2e-2, f"{n1}: rel err {rel:.3e}"


# ------------------------------------------------------------------ OPT
def _opt_models(dtype, p=0.0, lora_p=0.0):
    from mift.models.opt import OPTConfig, OPTForCausalLM
    cfg = OPTConfig(vocab_size=1000, hidden_size=320, num_hidden_layers=2, ffn_dim=1280, num_attention_heads=4,
                    max_position_embeddings=128, dropout=p)                     # head dim 80 (as OPT-2.7B)
    ref = OPTForCausalLM(cfg, dtype=torch.float32, device="cuda").init_weights(5)
    with torch.no_grad():  # same (rounded) base weights on both sides: only compute precision differs
        for q in ref.parameters():
            q.copy_(q.to(dtype).float())
    tm = ["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"]
    L.inject(ref, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=lora_p, target_modules=tm))
    for _, q in L.lora_parameters(ref):
        with torch.no_grad():
            q.normal_(0, 0.05)
    fused = copy.deepcopy(ref)
    for n, q in fused.named_parameters():
        if "lora_" not in n:
            q.data = q.data.to(dtype)
    ref.fused = False
    return cfg, ref, fused


def _grad_close(ma, mb, tol):
    for (n1, p1), (n2, p2) in zip(L.lora_parameters(ma), L.lora_parameters(mb)):
        g1, g2 = p1.grad.float(), p2.grad.float()
        rel = (g1 - g2).norm() / (g1.norm() + 1e-6)
        assert rel < tol, f"{n1}: rel err {rel:.3e}"


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_opt_fused_matches_reference(dtype, p):
    """Dropout masks are counter-hash generated, so ref and fused agree even with dropout on."""
    cfg, ref, fused = _opt_models(dtype, p, lora_p=0.05 if p else 0.0)
    torch.manual_seed(1)
    ids = torch.randint(3, cfg.vocab_size, (3, 96), device="cuda")
    mask = torch.ones_like(ids)
    mask[1, 70:] = 0
    ids[1, 70:] = 1
    ref.train()
    fused.train()
    lr = ref(input_ids=ids, attention_mask=mask, labels=ids, ignore_index=1, reduction="sum")["loss"]
    lr.backward()
    lf = fused(input_ids=ids, attention_mask=mask, labels=ids, ignore_index=1, reduction="sum")["loss"]
    lf.backward()
    torch.testing.assert_close(lf.float(), lr.float(), rtol=2e-2, atol=1e-1)
    # measured: fp16 1-4 %, bf16 3-9 % rel — 16-bit arithmetic itself (PyTorch's 16-bit eager path is
    # as far from fp32: test_opt_fused_grads_as_accurate_as_torch_16bit); the same with and without
    # dropout, i.e. the masks agree exactly
    _grad_close(ref, fused, 5e-2 if dtype == torch.float16 else 1.2e-1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_opt_fused_grads_as_accurate_as_torch_16bit(dtype):
    """The fused-vs-fp32 gradient gap is 16-bit arithmetic itself, not a kernel defect: PyTorch's own
    16-bit eager path on the same (rounded) weights — matmuls, SDPA, ReLU in bf16/fp16 — is as far
    from the fp32 reference, and the fused kernels stay within 1.25x of it (+1 % absolute) on every
    LoRA tensor.  The earlier "ReLU-kink flips" explanation did not hold: pushing fc1
    pre-activations away from 0 (bias +-1/2/4, tools/diag_opt_relu.py) made the bf16 gap larger,
    not smaller (6 % -> 21 % -> 69 % on layer-1 q/k), with no pre-activation near the kink — the gap
    follows the attention-backward cancellation dS = P*(dP - D) at 16-bit P."""
    cfg, ref, fused = _opt_models(dtype, 0.0, lora_p=0.0)
    t16 = copy.deepcopy(fused)
    t16.fused = False  # PyTorch 16-bit eager ops, same weights as the fused model
    torch.manual_seed(1)
    ids = torch.randint(3, cfg.vocab_size, (3, 96), device="cuda")
    for m_ in (ref, fused, t16):
        m_.train()
        m_(input_ids=ids, labels=ids, reduction="sum")["loss"].backward()
    worst = []
    for (n, p32), (_, pf), (_, pt) in zip(L.lora_parameters(ref), L.lora_parameters(fused), L.lora_parameters(t16)):
        g = p32.grad.float()
        ef = float((pf.grad.float() - g).norm() / (g.norm() + 1e-6))
        et = float((pt.grad.float() - g).norm() / (g.norm() + 1e-6))
        worst.append((ef, et, n))
        assert ef <= 1.25 * et + 1e-2, f"{n}: fused rel err {ef:.3e} vs torch 16-bit {et:.3e}"
    print(sorted(worst, reverse=True)[:3])


def test_opt_arena_multi_adapter_matches_dense():
    from mift.lora import LoraArena
    from mift.lora.pack import attach
    cfg, ref, fused = _opt_models(torch.float16, 0.1, 0.05)
    fused2 = copy.deepcopy(fused)
    ids = torch.randint(3, cfg.vocab_size, (2, 128), device="cuda")
    fused.train()
    fused2.train()
    fused(input_ids=ids, labels=ids, reduction="sum")["loss"].backward()
    arena = LoraArena(fused2)
    attach(fused2, arena, torch.float16)
    fused2(input_ids=ids, labels=ids, reduction="sum")["loss"].backward()
    arena.rebind_grads()
    _grad_close(fused, fused2, 2e-2)


def test_pack_lora_multi_matches_torch_pack():
    """The per-step one-launch pack of the q/k/v adapter group (pack_lora_multi, LoraPack.multi) writes
    exactly the operands the torch-op construction of MultiAdapterOps builds (s·A rows, B row spans,
    s·Bᵀ, Aᵀ; zeros elsewhere), for fp16 and bf16."""
    from mift.lora import LoraArena
    from mift.lora.pack import attach
    from mift.ops.fused import MultiAdapterOps
    for dt in (torch.float16, torch.bfloat16):
        cfg, ref, fused = _opt_models(dt, 0.1, 0.05)
        arena = LoraArena(fused)
        with torch.no_grad():
            arena.param.copy_(torch.randn_like(arena.param))
        cat = fused.model.decoder.layers[1].self_attn.qkv
        a = MultiAdapterOps(cat, dt)  # no pack attached: torch ops
        attach(fused, arena, dt)
        cat._mpack = None
        b = MultiAdapterOps(cat, dt)  # LoraPack.multi
        for x, y in ((a.A32s, b.A32s), (a.B32, b.B32), (a.B32t, b.B32t), (a.At32, b.At32)):
            assert x.shape == y.shape and torch.equal(x, y)


def test_fused_backward_notifies_dp_reducer_per_layer(monkeypatch):
    """DDP overlap on the fused path (mift.ops.fused._notify -> arena.grad_ready, which the DP
    reducer turns into bucket all-reduces): a fake reducer records the order of notifications
    against the dgrad GEMMs.  Layer l's adapters must be reported final BEFORE layer l-1's dgrad
    GEMMs are queued — otherwise no all-reduce could overlap the rest of backward."""
    import re
    from mift.lora import LoraArena
    from mift.lora.pack import attach
    from mift.ops import fused as F
    cfg = GPT2Config(vocab_size=1000, n_positions=128, n_embd=128, n_layer=4, n_head=2, n_inner=512,
                     embd_pdrop=0.0, attn_pdrop=0.0, resid_pdrop=0.0)
    model = GPT2LMHeadModel(cfg, dtype=torch.bfloat16, device="cuda").init_weights(3)
    L.inject(model, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0, target_modules=["c_attn", "c_proj"]))
    arena = LoraArena(model)
    attach(model, arena, torch.bfloat16)
    layer_of = {}
    for (n, _), off in zip(arena.named, arena.offsets):
        layer_of[off] = int(re.search(r"\.h\.(\d+)\.", n).group(1))
    events = []
    arena.grad_ready = lambda offs: events.append(("notify", {layer_of[o] for o in offs}))
    real_gemm = F.K.gemm

    def gemm(*a, **k):
        events.append(("gemm", None))
        return real_gemm(*a, **k)

    monkeypatch.setattr(F.K, "gemm", gemm)
    model.train()
    ids = torch.randint(0, cfg.vocab_size, (4, 64), device="cuda")
    loss = model(input_ids=ids, labels=ids, reduction="sum")["loss"]
    events.clear()  # forward GEMMs are not of interest
    loss.backward()
    torch.cuda.synchronize()
    notes = [(i, ls) for i, (kind, ls) in enumerate(events) if kind == "notify"]
    seen = set().union(*[ls for _, ls in notes])
    assert seen == set(range(cfg.n_layer)), seen
    order = [max(ls) for _, ls in notes]
    assert order == sorted(order, reverse=True), order  # last layer first
    last_of = {}
    for i, ls in notes:
        for l in ls:
            last_of[l] = i
    for l in range(cfg.n_layer - 1, 0, -1):
        # a dgrad GEMM of an earlier layer runs AFTER layer l's final notification
        assert any(kind == "gemm" for kind, _ in events[last_of[l] + 1:]), (l, events)
    # and the arena grads are the real ones (non-zero)
    assert arena.grad.abs().sum().item() > 0


def test_ln_backward_handoff_fires_and_matches_separate_passes(monkeypatch):
    """GradHandoff: at D = 768 every LN backward that feeds a LoRA linear's residual-dropout backward runs
    them as one pass (ln_bwd_mask_proj: the MLP's LN for attn.c_proj in every block, the next block's
    ln_1 — or the head's ln_f — for mlp.c_proj), and the LoRA gradients match the separate LN-bwd + mask_proj passes."""
    from mift.ops import kernels as K
    cfg = GPT2Config(vocab_size=1000, n_positions=128, n_embd=768, n_layer=3, n_head=12, n_inner=3072,
                     embd_pdrop=0.1, attn_pdrop=0.1, resid_pdrop=0.1)
    m = GPT2LMHeadModel(cfg, dtype=torch.bfloat16, device="cuda").init_weights(5)
    L.inject(m, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=["c_attn", "c_proj"]))
    for _, p in L.lora_parameters(m):
        with torch.no_grad():
            p.normal_(0, 0.05)
    m.train()
    ids = torch.randint(0, cfg.vocab_size, (4, 128), device="cuda")
    calls = []
    orig = K.ln_bwd_mask_proj
    monkeypatch.setattr(K, "ln_bwd_mask_proj", lambda *a, **k: calls.append(1) or orig(*a, **k))

    def grads(on):
        monkeypatch.setenv("MIFT_LN_MASK_PROJ", "1" if on else "0")
        for _, p in L.lora_parameters(m):
            p.grad = None
        m.micro_step = 3
        m(input_ids=ids, labels=ids, reduction="sum")["loss"].backward()
        return [p.grad.float().clone() for _, p in L.lora_parameters(m)]

    g1 = grads(True)
    assert len(calls) == 2 * cfg.n_layer, len(calls)  # + the final LN's (fused LM head) for the last mlp
    g0 = grads(False)
    assert len(calls) == 2 * cfg.n_layer
    for a, b in zip(g1, g0):
        rel = (a - b).norm() / (b.norm() + 1e-6)
        assert rel < 2e-2, rel
