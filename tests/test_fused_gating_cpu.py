"""Host-side dispatch rules of the fused path (no GPU): which widths take the MFMA row passes, the
chunked LM head's chunk size, the decode LN-fold cache keying, and the generate() host mask checks."""
import pytest
import torch

from mift.ops import fused as F


@pytest.mark.parametrize("D,kind,exp", [(768, "ln", True), (1024, "ln_bwd", True), (2560, "ln", True),
                                        (2560, "ln_bwd", True), (4096, "ln", False), (4096, "ln_bwd", False),
                                        (4096, "mask", True), (2048, "mask", True), (1536, "mask", False),
                                        (3072, "ln", False)])
def test_mfma_row_pass_widths(D, kind, exp, monkeypatch):
    monkeypatch.delenv("MIFT_ROWPROJ_WIDE", raising=False)
    assert F._mfma_width(D, kind) is exp
    monkeypatch.setenv("MIFT_ROWPROJ_WIDE", "0")  # A/B knob: only the round-4 widths
    assert F._mfma_width(D, kind) is (D in (768, 1024))


def test_row_kernel_fallback_for_narrow_rank(monkeypatch):
    monkeypatch.delenv("MIFT_ROWPROJ_WIDE", raising=False)
    assert F._rowproj_fused(512, 8, "ln")        # one-wave-per-row kernel, few rows, D <= 1024
    assert not F._rowproj_fused(512, 24, "ln")   # too many rows for the VALU row kernel
    assert not F._rowproj_fused(3072, 8, "mask")


@pytest.mark.parametrize("M,shift,env,exp", [(8192, 256, "0", 0), (8192, 256, "2048", 2048), (8192, 256, "1000", 768),
                                             (8192, 256, "100", 256), (8192, 0, "3000", 3000), (8192, 256, "8192", 0),
                                             (8192, 0, "9000", 0)])
def test_lm_chunk_rows(M, shift, env, exp, monkeypatch):
    """Chunks hold whole sequences when the labels are unshifted ids, and only exist when they split M."""
    monkeypatch.setenv("MIFT_LM_CHUNK", env)
    assert F._lm_chunk(M, shift) == exp


def test_ln_fold_cache_follows_in_place_updates():
    """The decode LN fold (wf = γ∘w, c1, c2) is rebuilt after any in-place update of its operands and
    equals LayerNorm followed by the linear (CPU arithmetic check of the algebra)."""
    torch.manual_seed(0)
    K, N = 64, 48
    ln = torch.nn.LayerNorm(K)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)

    class Lin:
        pass

    lin = Lin()
    w = torch.randn(N, K) / K ** 0.5
    lin.bias = torch.randn(N) * 0.1
    x = torch.randn(5, K) * 3 + 1
    wf, c1, c2 = F._ln_fold(ln, lin, w)
    mean = x.mean(1, keepdim=True)
    rstd = (x.var(1, unbiased=False, keepdim=True) + ln.eps).rsqrt()
    y = rstd * (x @ wf.t() - mean * c1) + c2
    ref = torch.nn.functional.linear(ln(x), w, lin.bias)
    torch.testing.assert_close(y, ref, atol=1e-4, rtol=1e-4)
    assert F._ln_fold(ln, lin, w)[0] is wf  # cached
    with torch.no_grad():
        ln.bias.add_(0.5)
    wf2, c12, c22 = F._ln_fold(ln, lin, w)
    assert not torch.equal(c22, c2)
    ref2 = torch.nn.functional.linear(ln(x), w, lin.bias)
    torch.testing.assert_close(rstd * (x @ wf2.t() - mean * c12) + c22, ref2, atol=1e-4, rtol=1e-4)


def test_generate_rejects_right_padding():
    """generate()'s host-side mask checks: left padding only (HF padding_side='left')."""
    from mift.infer.generate import generate
    from mift.models.gpt2 import GPT2Config, GPT2LMHeadModel
    m = GPT2LMHeadModel(GPT2Config(vocab_size=100, n_positions=32, n_embd=32, n_layer=1, n_head=2, n_inner=64),
                        dtype=torch.float32, device="cpu").init_weights(1)
    ids = torch.randint(0, 100, (2, 6))
    right = torch.tensor([[1, 1, 1, 1, 0, 0], [1, 1, 1, 1, 1, 1]])
    with pytest.raises(ValueError, match="left padding"):
        generate(m, ids, attention_mask=right, max_new_tokens=3)
    left = torch.tensor([[0, 0, 1, 1, 1, 1], [1, 1, 1, 1, 1, 1]])
    out = generate(m, ids, attention_mask=left, max_new_tokens=3, eos_token_id=-1)
    assert out.shape == (2, 9) and torch.equal(out[:, :6], ids)


def test_arena_version_follows_bumps_and_new_arenas():
    """The graphed generate() key reads the arena through a remembered module (no module walk per
    call): it follows version bumps and a NEW arena bound to the same model, and None without one."""
    from mift import lora as L
    from mift.infer import generate as G
    from mift.models import build_causal_lm
    m = build_causal_lm("opt-tiny", dtype=torch.float32, seed=0)
    assert G._arena_version(m) is None
    L.inject(m, L.LoraConfig(r=8, lora_alpha=16, target_modules=["q_proj", "v_proj"]))
    a = L.LoraArena(m)
    assert G._arena_version(m) == (id(a), 0)
    a.bump()
    assert G._arena_version(m) == (id(a), 1)
    b = L.LoraArena(m)
    assert G._arena_version(m) == (id(b), 0)
