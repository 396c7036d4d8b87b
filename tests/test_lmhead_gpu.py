"""Fused LM head + cross-entropy (csrc/kernels/gemm.hip EPI 1/2, ops.fused.LMHeadXent) vs a plain
PyTorch fp32 reference: loss, per-row logsumexp and the gradient w.r.t. the hidden states, for
both vocab sizes (GPT-2 50257, OPT 50272 padded to 50304), bf16 and fp16, with ignored targets
(-100 and OPT's pad-id ignore_index), and an upstream gradient that is not 1."""
import pytest
import torch
import torch.nn.functional as TF

import mift
from mift.ops import fused as F
from mift.ops import kernels as K

pytestmark = pytest.mark.gpu


class _LN(torch.nn.Module):
    def __init__(self, d, dtype, dev, g):
        super().__init__()
        self.weight = torch.nn.Parameter((1 + 0.1 * torch.randn(d, generator=g, device=dev)).to(dtype),
                                         requires_grad=False)
        self.bias = torch.nn.Parameter((0.1 * torch.randn(d, generator=g, device=dev)).to(dtype), requires_grad=False)
        self.eps = 1e-5


def _case(V, dtype, ignore_index, M=1536, d=768, scale=1.0):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(V + M)
    Vp = (V + 63) // 64 * 64
    h = torch.randn(M, d, generator=g, device=dev).to(dtype)
    ln = _LN(d, dtype, dev, g)
    W = torch.zeros(Vp, d, device=dev, dtype=dtype)
    W[:V] = (scale * 0.05 * torch.randn(V, d, generator=g, device=dev)).to(dtype)
    lab = torch.randint(0, V, (M,), generator=g, device=dev)
    lab[::7] = ignore_index
    if ignore_index >= 0:
        lab[3] = ignore_index
    return h, ln, W, lab, Vp


def _ref(h, ln, W, lab, V, ignore_index, gup):
    hf = h.float().requires_grad_(True)
    a = TF.layer_norm(hf, (hf.shape[1],), ln.weight.float(), ln.bias.float(), ln.eps)
    logits = a @ W[:V].float().t()
    loss = TF.cross_entropy(logits, lab, ignore_index=ignore_index, reduction="sum")
    (loss * gup).backward()
    lse = torch.logsumexp(logits, dim=1)
    return loss.detach(), hf.grad, lse.detach()


@pytest.mark.parametrize("V,dtype,ignore", [(50257, torch.bfloat16, -100), (50272, torch.float16, 1),
                                            (50257, torch.float16, -100), (50272, torch.bfloat16, 1)])
def test_fused_lmhead_matches_fp32(V, dtype, ignore):
    assert mift.kernels_available()
    h, ln, W, lab, Vp = _case(V, dtype, ignore)
    gup = 0.37
    hx = h.clone().requires_grad_(True)
    loss = F.lm_head_xent(hx, ln, W, lab, V, ignore, need_grad=True, w_kn=W.t().contiguous())
    (loss * gup).backward()
    rl, rg, rlse = _ref(h, ln, W, lab, V, ignore, gup)
    assert float(loss.detach()) == pytest.approx(float(rl), rel=3e-3)
    err = (hx.grad.float() - rg).norm() / rg.norm()
    assert err < 3e-2, float(err)


def test_lmhead_stats_and_lse():
    """Kernel pieces: E = exp(z - m_tile) <= 1, tile max, per-row lse, label logit."""
    V, dtype = 50257, torch.bfloat16
    h, ln, W, lab, Vp = _case(V, dtype, -100, M=512)
    a, _, _ = K.layer_norm_fwd(h, ln.weight, ln.bias, ln.eps)
    E, stats, lse, loss, zlab = K.lmhead_fwd(a, W, lab, V)
    z = a.float() @ W.float().t()
    zr = z[:, :V]
    assert E.shape == (512, Vp) and stats.shape == (512, (Vp + 255) // 256, 2)
    torch.testing.assert_close(lse, torch.logsumexp(zr, 1), atol=2e-2, rtol=1e-3)
    m_ref = torch.stack([zr[:, j * 256:min(V, (j + 1) * 256)].max(1).values for j in range(stats.shape[1])], 1)
    torch.testing.assert_close(stats[..., 0], m_ref, atol=2e-2, rtol=1e-3)
    Ef = E.float()[:, :V]
    assert float(Ef.max()) <= 1.0 + 1e-3 and float(E.float()[:, V:].abs().max()) == 0.0
    tm = stats[..., 0].repeat_interleave(256, 1)[:, :V]
    torch.testing.assert_close(Ef, torch.exp(zr - tm), atol=1e-2, rtol=1e-2)
    ok = lab >= 0
    torch.testing.assert_close(zlab[ok], zr[ok].gather(1, lab[ok, None])[:, 0], atol=2e-2, rtol=1e-3)
    torch.testing.assert_close(loss[~ok], torch.zeros_like(loss[~ok]))


def test_lmhead_large_logits_stable():
    """Peaked rows (|z| ~ 60): tile-relative E keeps every value finite and the loss exact."""
    V, dtype = 50257, torch.bfloat16
    h, ln, W, lab, Vp = _case(V, dtype, -100, M=768, scale=6.0)
    hx = h.clone().requires_grad_(True)
    loss = F.lm_head_xent(hx, ln, W, lab, V, -100, need_grad=True, w_kn=W.t().contiguous())
    loss.backward()
    rl, rg, _ = _ref(h, ln, W, lab, V, -100, 1.0)
    assert torch.isfinite(hx.grad).all()
    assert float(loss.detach()) == pytest.approx(float(rl), rel=3e-3)
    assert float((hx.grad.float() - rg).norm() / rg.norm()) < 3e-2


@pytest.mark.parametrize("V,dtype,ignore", [(50257, torch.bfloat16, -100), (50272, torch.float16, 1)])
def test_lmhead_in_kernel_shift(V, dtype, ignore):
    """shift = S (labels passed unshifted, the causal shift done by the kernels) equals the
    host-shifted labels, loss and gradient, incl. OPT's pad-id ignore index."""
    from mift.models.base import shift_labels
    S = 128
    h, ln, W, lab, Vp = _case(V, dtype, ignore, M=4 * S)
    gup = 0.5
    ids = lab.view(4, S)
    hx = h.clone().requires_grad_(True)
    loss = F.lm_head_xent(hx, ln, W, ids, V, ignore, need_grad=True, w_kn=W.t().contiguous(), shift=S)
    (loss * gup).backward()
    rl, rg, _ = _ref(h, ln, W, shift_labels(ids, ignore).reshape(-1), V, ignore, gup)
    assert float(loss.detach()) == pytest.approx(float(rl), rel=3e-3)
    assert float((hx.grad.float() - rg).norm() / rg.norm()) < 3e-2


def test_lmhead_in_launch_total_ignore_and_gmul():
    """The hygiene folds: the loss total reduced inside the lse launch equals the
    per-row sum and is bit-stable; the in-kernel ignore id equals masking the labels to -1 first;
    a gradient multiplier gmul gives the bits of the pre-multiplied fp32 upstream gradient."""
    V, dtype, ign = 50272, torch.float16, 1
    h, ln, W, lab, Vp = _case(V, dtype, ign, M=1024)
    a, _, _ = K.layer_norm_fwd(h, ln.weight, ln.bias, ln.eps)
    assert mift._ext.require().arrive_ints() == K.ARRIVE_INTS
    ws = torch.zeros(K.ARRIVE_INTS, dtype=torch.int32, device="cuda")
    outs = K.lmhead_fwd(a, W, lab, V, 0, ign, ws)
    E, stats, lse, loss, zlab, total = outs
    assert total.shape == (1,)
    assert float(total) == pytest.approx(float(loss.double().sum()), rel=1e-5)
    assert int(ws.abs().sum()) == 0  # counters reset by the arrivers
    bits = {tuple(K.lmhead_fwd(a, W, lab, V, 0, ign, ws)[5].view(torch.int32).tolist()) for _ in range(20)}
    assert len(bits) == 1
    masked = torch.where(lab == ign, torch.full_like(lab, -1), lab)
    E2, stats2, lse2, loss2, _ = K.lmhead_fwd(a, W, masked, V)
    assert torch.equal(loss, loss2) and torch.equal(lse, lse2) and torch.equal(E, E2)
    Wt = W.t().contiguous()
    s = torch.tensor([1024.0], device="cuda")
    m = torch.tensor([1.0 / 4093.0], device="cuda")
    d1 = K.lmhead_dgrad(E, Wt, W, lab, V, stats, lse, s, 0, ign, m)
    d2 = K.lmhead_dgrad(E, Wt, W, masked, V, stats, lse, s * m)
    assert torch.equal(d1, d2)


@pytest.mark.parametrize("V,dtype,ignore,shift", [(50257, torch.bfloat16, -100, 128), (50272, torch.float16, 1, 0)])
def test_lmhead_chunked_matches_whole(V, dtype, ignore, shift, monkeypatch):
    """MIFT_LM_CHUNK (SURVEY K7's chunked head: each chunk's E consumed by its dgrad inside forward, no
    [T, V] tensor kept): loss and gradient equal the fp32 reference and the whole-batch head, with a
    graph-style gradient multiplier (set_head_grad_mul) and a non-unit upstream gradient."""
    from mift.models.base import shift_labels
    M = 4 * 128
    h, ln, W, lab, Vp = _case(V, dtype, ignore, M=M)
    ids = lab.view(-1, 128) if shift else lab
    rlab = shift_labels(ids, ignore).reshape(-1) if shift else lab
    gmul = torch.full((1,), 0.25, device="cuda")
    res = {}
    for chunk in ("0", "256"):
        monkeypatch.setenv("MIFT_LM_CHUNK", chunk)
        hx = h.clone().requires_grad_(True)
        F.set_head_grad_mul(gmul)
        loss = F.lm_head_xent(hx, ln, W, ids, V, ignore, need_grad=True, w_kn=W.t().contiguous(), shift=shift)
        assert F.head_grad_mul_used()
        F.set_head_grad_mul(None)
        (loss * 2.0).backward()
        res[chunk] = (float(loss.detach()), hx.grad.float())
    rl, rg, _ = _ref(h, ln, W, rlab, V, ignore, 0.5)
    for chunk, (l, gr) in res.items():
        assert l == pytest.approx(float(rl), rel=3e-3), chunk
        assert float((gr - rg).norm() / rg.norm()) < 3e-2, chunk
    assert float((res["256"][1] - res["0"][1]).norm() / res["0"][1].norm()) < 1e-2
