"""Numerics of the HIP kernels vs the fp32 PyTorch reference (mift.ops.reference)."""
import pytest
import torch

import mift
from mift.ops import reference as ref

pytestmark = pytest.mark.gpu



def _gnt(C, *args):
    """gemm_nt with the epilogue projection off -> (out, preact)."""
    return C.gemm_nt(*args, None, 32, 0.0, 0)[:2]

def _C():
    assert mift.kernels_available(), f"extension not loaded: {mift._ext.error()!r}"
    import mift._C as C
    return C


@pytest.mark.parametrize("D", [64, 768, 2560, 4096])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_layer_norm_fwd_bwd(D, dt):
    C = _C()
    torch.manual_seed(0)
    M = 300
    x = torch.randn(M, D, device="cuda", dtype=dt)
    w = (1 + 0.1 * torch.randn(D, device="cuda")).to(dt)
    b = (0.1 * torch.randn(D, device="cuda")).to(dt)
    y, mean, rstd = C.layer_norm_fwd(x, w, b, 1e-5)
    xr = x.float().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (D,), w.float(), b.float(), 1e-5)
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    dy = torch.randn_like(x)
    dres = torch.randn_like(x)
    yr.backward(dy.float())
    dx, dbr, dw, db = C.layer_norm_bwd(dy, x, w, mean, rstd, dres, True, 0.1, 1234, False)
    exp = xr.grad + dres.float()
    torch.testing.assert_close(dx.float(), exp, atol=5e-2, rtol=3e-2)
    mask = ref.keep_mask(1234, (M, D), 0.1, device="cuda")
    torch.testing.assert_close(dbr.float(), torch.where(mask, dx.float() / 0.9, torch.zeros_like(exp)),
                               atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1000, 2304, 768), (8192, 768, 3072), (130, 200, 128)])
def test_gemm_nt_plain(M, N, K):
    C = _C()
    torch.manual_seed(1)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    out = _gnt(C, a, b, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0)[0]
    exp = a.float() @ b.float().t()
    torch.testing.assert_close(out.float(), exp, atol=3e-2, rtol=2e-2)


def test_gemm_nt_identity_asymmetric():
    """A = I with an asymmetric B catches swapped C/D layouts (guide §3)."""
    C = _C()
    n = 128
    a = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    bm = (torch.arange(n * n, device="cuda", dtype=torch.float32).view(n, n) % 97).to(torch.bfloat16)
    out = _gnt(C, a, bm, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0)[0]
    torch.testing.assert_close(out.float(), bm.float().t())


@pytest.mark.parametrize("act", [1, 2])
def test_gemm_nt_fused_epilogue(act):
    C = _C()
    torch.manual_seed(2)
    M, N, K = 512, 384, 256
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    a2 = torch.randn(M, 32, device="cuda", dtype=torch.bfloat16)
    b2 = torch.randn(N, 32, device="cuda", dtype=torch.bfloat16) * 0.1
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    out, pre = _gnt(C, a, b, bias, a2, b2, act, None, res, 0.1, 77, True, 1.0, None, 0, None, None, 0.0, 0)
    exp, exp_pre = ref.gemm_nt(a, b, bias, a2, b2, act, None, res, 0.1, 77, True)
    torch.testing.assert_close(pre.float(), exp_pre.float(), atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(out.float(), exp.float(), atol=8e-2, rtol=3e-2)


@pytest.mark.parametrize("act", [4, 5])
def test_gemm_nt_act_backward(act):
    C = _C()
    torch.manual_seed(3)
    M, N, K = 256, 512, 128
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    aux = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    out = _gnt(C, a, b, None, None, None, act, aux, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0)[0]
    exp, _ = ref.gemm_nt(a, b, None, None, None, act, aux)
    torch.testing.assert_close(out.float(), exp.float(), atol=5e-2, rtol=3e-2)


@pytest.mark.parametrize("V,ldV,dtype", [(1000, 1024, torch.bfloat16), (50257, 50304, torch.bfloat16),
                                         (50272, 50272, torch.float16), (3000, 3008, torch.float16)])
def test_xent_fwd_bwd(V, ldV, dtype):
    C = _C()
    torch.manual_seed(4)
    M = 64
    logits = (torch.randn(M, ldV, device="cuda") * 3).to(dtype)
    labels = torch.randint(0, V, (M,), device="cuda")
    labels[::7] = -100
    labels[1], labels[2] = V - 1, 0  # first / last column (tail chunk)
    x = logits[:, :V].float().requires_grad_(True)
    ref_loss = torch.nn.functional.cross_entropy(x, labels, ignore_index=-100, reduction="none")
    ref_loss.sum().backward()
    buf = logits.clone()
    loss, lse = C.xent_fwd_bwd(buf, labels, V, -100, True)
    torch.testing.assert_close(loss, ref_loss.detach(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(buf[:, :V].float(), x.grad, atol=1e-2, rtol=2e-2)
    assert (buf[:, V:] == 0).all()


def test_adamw_matches_torch():
    C = _C()
    torch.manual_seed(5)
    n = 10_000
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda") * 3.0
    from mift.train.optim import FusedAdamW
    pt = p.clone().requires_grad_(True)
    ref = torch.optim.AdamW([pt], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    opt = FusedAdamW(p, g.clone(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    for _ in range(3):
        gg = g.clone()
        opt.g.copy_(gg)
        opt.step()
        pt.grad = gg.clone()
        torch.nn.utils.clip_grad_norm_([pt], 1.0)
        ref.step()
    torch.testing.assert_close(opt.p, pt.detach(), atol=1e-5, rtol=1e-4)
    assert opt.g.abs().max().item() == 0.0


def test_mask_scale_and_embed():
    C = _C()
    x = torch.randn(1000, 64, device="cuda", dtype=torch.bfloat16)
    y = C.mask_scale(x, 0.1, 99, None, False)
    exp = ref.dropout(x.float(), 0.1, 99)
    torch.testing.assert_close(y.float(), exp, atol=1e-2, rtol=1e-2)
    wte = torch.randn(500, 64, device="cuda", dtype=torch.bfloat16)
    wpe = torch.randn(128, 64, device="cuda", dtype=torch.bfloat16)
    ids = torch.randint(0, 500, (4, 32), device="cuda")
    h = C.embed_fwd(ids, None, wte, wpe, 0, 0.0, 0, torch.bfloat16)
    e = (wte[ids].float() + wpe[torch.arange(32, device="cuda")][None].float()).view(-1, 64)
    torch.testing.assert_close(h.float(), e, atol=2e-2, rtol=1e-2)


def _attn_ref(qkv, B, S, H, hd, scale, p, seed, kv_len=None):
    q, k, v = qkv.float().view(B, S, 3, H, hd).unbind(2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    valid = None
    if kv_len is not None:
        valid = torch.arange(S, device=qkv.device)[None, :] < kv_len[:, None]
    o = ref.attention(q, k, v, causal=True, key_padding=valid, scale=scale, dropout_p=p, seed=seed)
    return o.transpose(1, 2).reshape(B * S, H * hd)


@pytest.mark.parametrize("hd", [64, 80, 128])
@pytest.mark.parametrize("S", [256, 200])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_flash_attention_fwd_bwd(hd, S, p, dt):
    C = _C()
    torch.manual_seed(6)
    B, H = 2, 3
    scale = hd ** -0.5
    qkv = (torch.randn(B * S, 3 * H * hd, device="cuda")).to(dt)
    o, lse = C.attn_fwd(qkv, B, S, H, hd, scale, p, 321, None)
    x = qkv.float().requires_grad_(True)
    oref = _attn_ref(x, B, S, H, hd, scale, p, 321)
    torch.testing.assert_close(o.float(), oref, atol=3e-2, rtol=3e-2)
    do = torch.randn_like(o)
    oref.backward(do.float())
    dqkv = C.attn_bwd(do, qkv, o, lse, B, S, H, hd, scale, p, 321, None)
    g = x.grad.view(B * S, 3, H * hd)
    dq = dqkv.float().view(B * S, 3, H * hd)
    for i, name in enumerate("qkv"):
        err = (dq[:, i] - g[:, i]).norm() / (g[:, i].norm() + 1e-6)
        assert err < 3e-2, f"d{name} rel err {err:.3e}"


@pytest.mark.parametrize("S", [256, 200])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_flash_attention_whole_sequence_kernels(S, p, dt, monkeypatch):
    """The whole-sequence-in-LDS kernels (MIFT_ATTN_SEQ=2 forces them at this small head count)
    against the fp32 reference, and bit-for-bit agreement of fwd with the tiled kernel."""
    monkeypatch.setenv("MIFT_ATTN_SEQ", "2")
    test_flash_attention_fwd_bwd(64, S, p, dt)
    C = _C()
    B, H, hd = 2, 3, 64
    qkv = torch.randn(B * S, 3 * H * hd, device="cuda").to(dt)
    kvl = torch.tensor([S - 37, S // 3], device="cuda", dtype=torch.int32)
    # same P·V operand order on both sides (the seq kernel defaults to the transposed-output MFMA,
    # the tiled one to the plain order: MFMA-internal summation order differs by an ulp in fp16)
    monkeypatch.setenv("MIFT_ATTN_OT", "1")
    o_seq, lse_seq = C.attn_fwd(qkv, B, S, H, hd, hd ** -0.5, p, 99, kvl)
    monkeypatch.setenv("MIFT_ATTN_SEQ", "0")
    o_til_ot, lse_til_ot = C.attn_fwd(qkv, B, S, H, hd, hd ** -0.5, p, 99, kvl)
    torch.testing.assert_close(o_seq, o_til_ot, atol=0, rtol=0)
    torch.testing.assert_close(lse_seq, lse_til_ot, atol=0, rtol=0)
    monkeypatch.delenv("MIFT_ATTN_OT")
    o_til, lse_til = C.attn_fwd(qkv, B, S, H, hd, hd ** -0.5, p, 99, kvl)
    torch.testing.assert_close(o_til, o_til_ot, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(lse_til, lse_til_ot, atol=0, rtol=0)
    do = torch.randn_like(o_til)
    d_til = C.attn_bwd(do, qkv, o_til, lse_til, B, S, H, hd, hd ** -0.5, p, 99, kvl)
    monkeypatch.setenv("MIFT_ATTN_SEQ", "2")
    d_seq = C.attn_bwd(do, qkv, o_til, lse_til, B, S, H, hd, hd ** -0.5, p, 99, kvl)
    torch.testing.assert_close(d_seq.float(), d_til.float(), atol=2e-3, rtol=2e-3)


@pytest.mark.parametrize("B,S", [(32, 256), (24, 200), (40, 256)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_head_split_bit_identical(B, S, p, monkeypatch):
    """C < B·H < 2C heads: the whole-sequence forward and dq kernels split 2C - B·H heads into two
    query ranges (one full + one half head per CU).  Every query's arithmetic is unchanged, so
    o, lse and dqkv equal the unsplit launch bit for bit (B = 40: 480 heads)."""
    monkeypatch.setenv("MIFT_ATTN_SEQ", "1")
    C = _C()
    torch.manual_seed(3)
    H, hd = 12, 64
    qkv = torch.randn(B * S, 3 * H * hd, device="cuda").to(torch.bfloat16)
    kvl = torch.randint(S // 2, S + 1, (B,), device="cuda", dtype=torch.int32)
    out = {}
    for split in ("1", "0"):
        monkeypatch.setenv("MIFT_ATTN_SPLIT", split)
        o, lse, bits = C.attn_fwd_bits(qkv, B, S, H, hd, hd ** -0.5, p, 5, kvl)
        torch.manual_seed(4)
        do = torch.randn_like(o)
        d = C.attn_bwd_bits(do, qkv, o, lse, B, S, H, hd, hd ** -0.5, p, 5, kvl, bits if bits.numel() else None)
        out[split] = (o, lse, bits, d)
    # o, lse, dqkv (the keep-bit record's never-visited, non-causal entries are left unwritten)
    for i, name in ((0, "o"), (1, "lse"), (3, "dqkv")):  # numerics vs fp32: test_flash_attention_*
        assert torch.equal(out["1"][i], out["0"][i]), name


@pytest.mark.parametrize("hd,S", [(64, 256), (64, 200), (32, 384), (80, 128), (128, 100)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_attention_keep_bits_match_hash(hd, S, dt, monkeypatch):
    """Dropout keep bits recorded by the whole-sequence forward (attn_fwd_bits) and read by the
    backward give exactly the re-hashing backward: same masks, same arithmetic -> equal dqkv."""
    monkeypatch.setenv("MIFT_ATTN_SEQ", "2")
    C = _C()
    torch.manual_seed(11)
    B, H, p = 2, 3, 0.1
    qkv = torch.randn(B * S, 3 * H * hd, device="cuda").to(dt)
    kvl = torch.tensor([S - 9, S // 3], device="cuda", dtype=torch.int32)
    for lens in (None, kvl):
        o, lse = C.attn_fwd(qkv, B, S, H, hd, hd ** -0.5, p, 77, lens)
        o2, lse2, bits = C.attn_fwd_bits(qkv, B, S, H, hd, hd ** -0.5, p, 77, lens)
        torch.testing.assert_close(o2, o, atol=0, rtol=0)
        torch.testing.assert_close(lse2, lse, atol=0, rtol=0)
        do = torch.randn_like(o)
        d_hash = C.attn_bwd(do, qkv, o, lse, B, S, H, hd, hd ** -0.5, p, 77, lens)
        d_bits = C.attn_bwd_bits(do, qkv, o, lse, B, S, H, hd, hd ** -0.5, p, 77, lens, bits if bits.numel() else None)
        torch.testing.assert_close(d_bits, d_hash, atol=0, rtol=0)
        if hd == 64:
            assert bits.numel() == B * H * S * ((S + 63) // 64 * 4)  # the record exists on this path


def test_flash_attention_kv_len():
    C = _C()
    torch.manual_seed(7)
    B, S, H, hd = 2, 128, 2, 64
    qkv = torch.randn(B * S, 3 * H * hd, device="cuda").to(torch.bfloat16)
    kvl = torch.tensor([100, 37], device="cuda", dtype=torch.int32)
    o, lse = C.attn_fwd(qkv, B, S, H, hd, hd ** -0.5, 0.0, 0, kvl)
    oref = _attn_ref(qkv, B, S, H, hd, hd ** -0.5, 0.0, 0, kvl)
    torch.testing.assert_close(o.float(), oref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("p", [0.0, 0.05])
@pytest.mark.parametrize("K", [768, 2304, 3072, 2560, 4096, 7680])
@pytest.mark.parametrize("M,nz", [(1000, 8), (1000, 24), (24576, 8)])
def test_lora_proj_and_wgrad(p, K, M, nz):
    """lora_proj for every block geometry (16- and 32-row blocks, one or two 16-column tiles:
    non-zero rows 8 -> one tile, 24 -> two) incl. the tall OPT-size input that used to go to
    torch.mm, and lora_wgrad, vs the fp32 reference."""
    C = _C()
    torch.manual_seed(8)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(32, K, device="cuda", dtype=torch.bfloat16)
    w[:nz] = (torch.randn(nz, K, device="cuda") * 0.05).to(torch.bfloat16)
    out = C.lora_proj(x, w, 2.0, p, 55, nz)
    xd = ref.dropout(x.float(), p, 55)
    torch.testing.assert_close(out.float(), 2.0 * xd @ w.float().t(), atol=3e-2, rtol=3e-2)
    # K-split shapes reduce in the launch (per-row-block arrival counters, re-armed): same bits again
    assert torch.equal(C.lora_proj(x, w, 2.0, p, 55, nz), out)
    if M > 4096:
        return
    y = torch.randn(M, 32, device="cuda", dtype=torch.bfloat16)
    acc = torch.zeros(K, 32, device="cuda")
    C.lora_wgrad(x, y, acc, p, 55, 0, 32, 0, 0)
    exp = xd.t() @ y.float()
    err = (acc - exp).norm() / exp.norm()
    assert err < 1e-2, err


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_lora_wgrad_group(dt):
    """One grouped launch over a layer's worth of problems (kernels/lora.hip lora_wgrad_group):
    dB in [P, r] layout from a column slice of a wider gradient, a dropout-masked dA in [r, P]
    layout, a multi-slot dA (three adapters sharing one input, OPT q/k/v) and a ragged M —
    each against the fp32 reference, accumulated into one flat arena."""
    C = _C()
    torch.manual_seed(21)
    M, N, K = 1000, 3 * 256, 512
    gz = torch.randn(M, N, device="cuda", dtype=dt)
    x = torch.randn(M, K, device="cuda", dtype=dt)
    T = torch.randn(M, 32, device="cuda", dtype=dt)
    dT = torch.randn(M, 32, device="cuda", dtype=dt)
    xr = torch.randn(333, 128, device="cuda", dtype=dt)
    yr = torch.randn(333, 32, device="cuda", dtype=dt)
    arena = torch.zeros(200000, device="cuda")
    pad = [0, 0, 0] * 3
    meta, xs, ys, ps, exp = [], [], [], [], []
    # dB of the middle adapter: gz[:, 256:512], rank 8 at T columns 8..15 -> [256, 8] at offset 100
    xs.append(gz[:, 256:512]); ys.append(T); ps.append(0.0)
    meta += [1, 1, 8, 8, 100] + pad + [0]
    exp.append((100, (gz[:, 256:512].float().t() @ T.float()[:, 8:16]).reshape(-1)))
    # dA, dropout-masked input, rank 8 at columns 0..7 -> [8, K] at offset 5000
    xs.append(x); ys.append(dT); ps.append(0.05)
    meta += [2, 1, 0, 8, 5000] + pad + [77]
    xd = ref.dropout(x.float(), 0.05, 77)
    exp.append((5000, (xd.t() @ dT.float()[:, :8]).t().reshape(-1)))
    # multi-slot dA: three rank-4 adapters in columns 0, 10, 20 of one product
    xs.append(x); ys.append(dT); ps.append(0.0)
    meta += [2, 3, 0, 4, 20000, 10, 4, 30000, 20, 4, 40000, 0, 0, 0, 0]
    for q, off in [(0, 20000), (10, 30000), (20, 40000)]:
        exp.append((off, (x.float().t() @ dT.float()[:, q:q + 4]).t().reshape(-1)))
    # dense mode-0 problem with a ragged M
    xs.append(xr); ys.append(yr); ps.append(0.0)
    meta += [0, 1, 0, 32, 100000] + pad + [0]
    exp.append((100000, (xr.float().t() @ yr.float()).reshape(-1)))
    C.lora_wgrad_group(arena, xs, ys, meta, ps)
    covered = torch.zeros_like(arena, dtype=torch.bool)
    for off, e in exp:
        got = arena[off:off + e.numel()]
        err = (got - e).norm() / e.norm()
        assert err < 1e-2, (off, err.item())
        covered[off:off + e.numel()] = True
    assert arena[~covered].abs().max().item() == 0.0  # nothing written outside the slots


@pytest.mark.parametrize("det", ["1", "0"])
def test_lora_wgrad_group_deterministic(det, monkeypatch):
    """Deterministic mode (default): slab partials + ordered reduction, so repeated launches on the
    same inputs give ONE bit pattern; MIFT_DETERMINISTIC=0 (fp32 atomics) stays
    numerically correct."""
    monkeypatch.setenv("MIFT_DETERMINISTIC", det)
    C = _C()
    torch.manual_seed(5)
    M, K = 8192, 3072  # distilgpt2 mlp.c_proj dA: many row chunks per column tile
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    dT = torch.randn(M, 32, device="cuda", dtype=torch.bfloat16)
    meta = [2, 1, 0, 8, 64] + [0, 0, 0] * 3 + [9]
    outs = []
    for _ in range(5 if det == "1" else 1):
        arena = torch.full((64 + 8 * K + 64,), 0.25, device="cuda")  # accumulates onto existing grads
        C.lora_wgrad_group(arena, [x], [dT], meta, [0.05])
        outs.append(arena)
    exp = (ref.dropout(x.float(), 0.05, 9).t() @ dT.float()[:, :8]).t().reshape(-1) + 0.25
    got = outs[0][64:64 + 8 * K]
    assert ((got - exp).norm() / exp.norm()).item() < 1e-2
    assert outs[0][:64].eq(0.25).all() and outs[0][64 + 8 * K:].eq(0.25).all()
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), "deterministic wgrad must be bit-reproducible"


def test_grad_stats_deterministic():
    """grad_stats run 100x on the same arena gives one bit pattern (per-block partials + one
    fixed-order reduction block, no float atomics), close to the fp64 sum; non-finite count exact."""
    C = _C()
    g = torch.randn(11_796_481, device="cuda") * 1e-3  # OPT-2.7B LoRA arena size (+1: ragged tail)
    stats = torch.zeros(2, device="cuda")
    ref_s = (g.double() ** 2).sum().item()
    seen = set()
    for _ in range(100):
        C.grad_stats(g, stats)
        seen.add(tuple(stats.cpu().view(torch.int32).tolist()))
    assert len(seen) == 1, seen
    assert stats[0].item() == pytest.approx(ref_s, rel=1e-5)
    assert stats[1].item() == 0.0
    g[12345] = float("inf")
    g[-1] = float("nan")
    C.grad_stats(g, stats)
    assert stats[1].item() == 2.0


@pytest.mark.parametrize("rank,D", [(8, 768), (28, 768), (28, 2560), (8, 2560), (16, 1024), (8, 2048), (28, 4096),
                                    (8, 1536)])
@pytest.mark.parametrize("p", [0.0, 0.05])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_rowproj_fused_kernels(rank, D, p, dt):
    """LN fwd + LoRA projection and dropout-bwd + dT (csrc/kernels/rowproj.hip) vs fp32 reference.
    D in {768, 1024, 2048, 2560, 4096} runs the MFMA 16-row form on 4 / 8 / 16 waves (rank 28: two
    16-column output tiles), 1536 the one-wave-per-row form; M = 777 leaves a partial last 16-row tile."""
    C = _C()
    torch.manual_seed(11)
    M = 777
    x = torch.randn(M, D, device="cuda", dtype=dt)
    w = (1 + 0.1 * torch.randn(D, device="cuda")).to(dt)
    b = (0.1 * torch.randn(D, device="cuda")).to(dt)
    pw = torch.zeros(32, D, device="cuda", dtype=dt)
    pw[:rank] = (torch.randn(rank, D, device="cuda") * 0.05).to(dt)
    y, mean, rstd, t = C.layer_norm_fwd_proj(x, w, b, 1e-5, pw, rank, 1.5, p, 77)
    y0, m0, r0 = C.layer_norm_fwd(x, w, b, 1e-5)
    # same math as the plain LN kernel, row sums taken in a different order: <= 1 ulp of T apart
    ulp = 2.0 ** -7 if dt == torch.bfloat16 else 2.0 ** -10
    torch.testing.assert_close(y.float(), y0.float(), atol=ulp, rtol=ulp)
    torch.testing.assert_close(mean, m0, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rstd, r0, atol=1e-5, rtol=1e-5)
    yd = ref.dropout(y.float(), p, 77)
    torch.testing.assert_close(t.float(), 1.5 * yd @ pw.float().t(), atol=4e-2, rtol=3e-2)
    gz, dt_ = C.mask_proj(x, p, 99, pw, rank, 2.0)
    gexp = ref.dropout(x.float(), p, 99)
    torch.testing.assert_close(gz.float(), gexp, atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(dt_.float(), 2.0 * gz.float() @ pw.float().t(), atol=5e-2, rtol=3e-2)
    if p == 0.0:
        assert gz.data_ptr() == x.data_ptr()


def test_gemm_ext_masked():
    C = _C()
    torch.manual_seed(9)
    M, N, K = 512, 768, 256
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    a2 = torch.randn(M, 32, device="cuda", dtype=torch.bfloat16)
    b2 = torch.randn(N, 32, device="cuda", dtype=torch.bfloat16) * 0.1
    out = _gnt(C, a, b, None, a2, b2, 0, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.05, 1234)[0]
    exp = a.float() @ b.float().t() + ref.dropout(a2.float() @ b2.float().t(), 0.05, 1234)
    torch.testing.assert_close(out.float(), exp, atol=5e-2, rtol=3e-2)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10])
@pytest.mark.parametrize("M,N,K", [(4096, 2560, 2560), (2048, 2560, 1024), (1000, 2304, 768), (8192, 768, 3072), (777, 1000, 320),
                                   (300, 520, 64), (64, 2304, 768), (64, 768, 3072), (7, 3072, 768)])
def test_gemm_tiles_splitk_tail_fused(tile, M, N, K):
    """Every tile config incl. the split-K ragged-wave tail (triggered for these shapes on 256 CUs)
    and the small-grid split (decode shapes: every tile split into >= 2-k-tile chunks) with the
    full epilogue: bias, LoRA K-ext, gelu, pre-activation, dropout, residual."""
    C = _C()
    torch.manual_seed(11)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    a2 = torch.randn(M, 32, device="cuda", dtype=torch.bfloat16)
    b2 = torch.randn(N, 32, device="cuda", dtype=torch.bfloat16) * 0.1
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    out, pre = _gnt(C, a, b, bias, a2, b2, 1, None, res, 0.1, 5, True, 1.0, None, tile, None, None, 0.0, 0)
    exp, exp_pre = ref.gemm_nt(a, b, bias, a2, b2, 1, None, res, 0.1, 5, True)
    torch.testing.assert_close(pre.float(), exp_pre.float(), atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(out.float(), exp.float(), atol=8e-2, rtol=3e-2)
    # repeated calls re-use the self-re-arming tile counters
    out2 = _gnt(C, a, b, bias, a2, b2, 1, None, res, 0.1, 5, False, 1.0, None, tile, None, None, 0.0, 0)[0]
    assert torch.equal(out, out2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (256, 512, 128), (512, 256, 192), (1000, 704, 640),
                                   (2048, 2560, 2560), (777, 2304, 704)])
@pytest.mark.parametrize("epi", ["plain", "fwd", "relu_bits", "dgrad_masked", "gelu_pre"])
@pytest.mark.parametrize("pair", [(8, 10, "1"), (7, 7, "0"), (9, 9, "0"), (8, 8, "0"), (10, 10, "0")])
def test_gemm_4wave_tile_and_staged_epilogue_bit_identical(dt, M, N, K, epi, pair, monkeypatch):
    """(a) Tile 10 (4-wave 256x256 loop, one to three k-tiles through the steady state) accumulates every
    output element in the same MFMA order as tile 8: bit-identical outputs / pre-activations / sign
    bits for every epilogue family the training step uses.  (b) The feature-staged epilogue of interior
    tiles (default) against the per-chunk form (MIFT_EPI_STAGED=0) of the same tile: bit-identical."""
    ta, tb, staged_a = pair
    from mift.ops import kernels as K_
    C = _C()
    torch.manual_seed(3)
    a = torch.randn(M, K, device="cuda", dtype=dt)
    b = torch.randn(N, K, device="cuda", dtype=dt) / K ** 0.5
    bias = torch.randn(N, device="cuda", dtype=dt)
    a2 = torch.randn(M, 32, device="cuda", dtype=dt)
    b2 = torch.randn(N, 32, device="cuda", dtype=dt) * 0.1
    res = torch.randn(M, N, device="cuda", dtype=dt)
    aux = torch.randn(M, N, device="cuda", dtype=dt)

    def run(tile):
        if epi == "plain":
            return list(_gnt(C, a, b, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, tile, None, None, 0.0, 0))
        if epi == "fwd":
            return list(_gnt(C, a, b, bias, a2, b2, 0, None, res, 0.1, 5, False, 1.0, None, tile, None, None, 0.0, 0))
        if epi == "relu_bits":
            bits = torch.zeros(M, N // 8, dtype=torch.uint8, device="cuda")
            y = K_.gemm(a, b, bias, act=2, sbits=bits, tile=tile)
            return [y, bits]
        if epi == "dgrad_masked":
            return list(_gnt(C, a, b, None, a2, b2, 5, aux, None, 0.0, 0, False, 1.0, None, tile, None, None, 0.05, 77))
        return list(_gnt(C, a, b, bias, None, None, 1, None, None, 0.0, 0, True, 1.0, None, tile, None, None, 0.0, 0))

    monkeypatch.setenv("MIFT_EPI_STAGED", staged_a)
    o8 = run(ta)
    monkeypatch.setenv("MIFT_EPI_STAGED", "1")
    o10 = run(tb)
    for x, y in zip(o8, o10):
        if x is not None and x.numel():
            assert torch.equal(x, y)
    if epi == "plain":
        r = a.float() @ b.float().t()
        assert float((o10[0].float() - r).norm() / r.norm()) < 1e-2


@pytest.mark.parametrize("tile", [0, 3, 7, 8, 9, 10])
@pytest.mark.parametrize("rows,p", [(8, 0.0), (8, 0.05), (24, 0.05)])
def test_gemm_epilogue_projection_matches_lora_proj(tile, rows, p):
    """T = drop(out)·pwᵀ from the GEMM epilogue (per column tile partials in fp32 slabs, summed in
    order) == lora_proj over the stored output: same mask, fp32 sums, <= 16-bit rounding apart."""
    C = _C()
    torch.manual_seed(5)
    M, K, N = 1000, 256, 768 if tile == 7 else 3072
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    bias = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    pw = torch.zeros(32, N, device="cuda", dtype=torch.bfloat16)
    pw[:rows] = (0.05 * torch.randn(rows, N, device="cuda")).to(torch.bfloat16)
    out, pre, t = C.gemm_nt(a, b, bias, None, None, 1, None, None, 0.0, 0, True, 1.0, None, tile, None, None, 0.0, 0,
                            pw, rows, p, 4321)
    out0, pre0 = _gnt(C, a, b, bias, None, None, 1, None, None, 0.0, 0, True, 1.0, None, tile, None, None, 0.0, 0)
    assert torch.equal(out, out0) and torch.equal(pre, pre0)  # the projection leaves the GEMM output alone
    exp = C.lora_proj(out, pw, 1.0, p, 4321, rows)
    torch.testing.assert_close(t.float(), exp.float(), atol=2e-2, rtol=1e-2)
    assert float(t[:, rows if rows > 16 else 16:].abs().max()) == 0.0
    ref_t = ref.dropout(out.float(), p, 4321) @ pw.float().t()
    torch.testing.assert_close(t.float(), ref_t, atol=5e-2, rtol=3e-2)


@pytest.mark.parametrize("tile", [0, 8, 9, 10])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_dgrad_epilogue_projection_relu_bwd(tile, dt):
    """A dgrad GEMM with an activation-backward epilogue (ReLU-bwd on aux, OPT's fc2 dgrad) that also
    emits the next adapter's dT = alpha·out·pwᵀ (proj_alpha = the adapter scale) == lora_proj over its
    stored output; the GEMM output itself is unchanged by the projection."""
    from mift.ops import kernels as K_
    torch.manual_seed(6)
    M, K, N, rows, s = 1024, 512, 2560, 8, 2.0
    a = torch.randn(M, K, device="cuda").to(dt)
    b = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
    z = torch.randn(M, N, device="cuda").to(dt)
    pw = torch.zeros(32, N, device="cuda", dtype=dt)
    pw[:rows] = (0.05 * torch.randn(rows, N, device="cuda")).to(dt)
    out, t = K_.gemm(a, b, act=5, aux=z, tile=tile, proj_w=pw, proj_rows=rows, proj_alpha=s)
    out0 = K_.gemm(a, b, act=5, aux=z, tile=tile)
    assert torch.equal(out, out0)
    exp = K_.lora_proj(out, pw, s, 0.0, 0, rows=rows)
    torch.testing.assert_close(t.float(), exp.float(), atol=3e-2, rtol=1e-2)
    ref_t = s * out.float() @ pw.float().t()
    torch.testing.assert_close(t.float(), ref_t, atol=5e-2, rtol=3e-2)


@pytest.mark.parametrize("tile", [7, 8, 9, 10])
def test_nontemporal_c_stores_bit_identical(tile, monkeypatch):
    """MIFT_EPI_NT=1 (non-temporal C stores, the default for outputs >= 96 MiB) writes the same bits as
    the plain stores, with a residual-dropout epilogue and a ragged last column tile."""
    from mift.ops import kernels as K_
    torch.manual_seed(8)
    M, K, N = 1000, 512, 2560
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    bias = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    res = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    monkeypatch.setenv("MIFT_EPI_NT", "0")
    ref_out = K_.gemm(a, b, bias, residual=res, dropout_p=0.1, seed=3, tile=tile)
    monkeypatch.setenv("MIFT_EPI_NT", "1")
    out = K_.gemm(a, b, bias, residual=res, dropout_p=0.1, seed=3, tile=tile)
    assert torch.equal(out, ref_out)


@pytest.mark.parametrize("tile", [0, 7, 8, 9, 10])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_relu_sign_bits_roundtrip(tile, dt):
    """ReLU sign bits: the forward epilogue's bits are the packed (stored output > 0) mask (skinny-sized M
    included: the bits keep such GEMMs on the tiled path), and the ReLU backward reading them is
    bit-identical to the one reading the 16-bit output as aux — with the masked LoRA extension and the
    dT projection epilogue on top (OPT's fc2 dgrad)."""
    from mift.ops import kernels as K_
    torch.manual_seed(7)
    for M, K, N in ((1024, 512, 2560), (40, 256, 768)):
        a = torch.randn(M, K, device="cuda").to(dt)
        b = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
        bias = (0.1 * torch.randn(N, device="cuda")).to(dt)
        bits = torch.full((M, N // 8), 0xA5, dtype=torch.uint8, device="cuda")
        f = K_.gemm(a, b, bias, act=2, sbits=bits, tile=tile)
        # auto at M <= 64 without bits is the skinny kernel (another accumulation order): the tiled 64x64
        assert torch.equal(f, K_.gemm(a, b, bias, act=2, tile=4 if (tile == 0 and M <= 64) else tile))
        w8 = (1 << torch.arange(8, device="cuda", dtype=torch.int32))
        exp = ((f > 0).view(M, N // 8, 8).to(torch.int32) * w8).sum(-1).to(torch.uint8)
        assert torch.equal(bits, exp)
        g = torch.randn(M, K, device="cuda").to(dt)
        bt = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
        a2 = (0.1 * torch.randn(M, 32, device="cuda")).to(dt)
        b2 = (0.1 * torch.randn(N, 32, device="cuda")).to(dt)
        pw = torch.zeros(32, N, device="cuda", dtype=dt)
        pw[:8] = (0.05 * torch.randn(8, N, device="cuda")).to(dt)
        kw = dict(a2=a2, b2=b2, ext_p=0.05, ext_seed=11, act=5, tile=tile, proj_w=pw, proj_rows=8, proj_alpha=2.0)
        o1, t1 = K_.gemm(g, bt, aux=f, **kw)
        o2, t2 = K_.gemm(g, bt, sbits=bits, **kw)
        assert torch.equal(o1, o2) and torch.equal(t1, t2)


@pytest.mark.parametrize("M", [1, 7, 64])
@pytest.mark.parametrize("N,K", [(2304, 768), (768, 3072), (50304, 768), (3072, 768)])
def test_gemm_skinny_decode_shapes(M, N, K):
    """M <= 64: the skinny kernel for N <= 4096, K <= 1024 (blocks own 16 columns for all rows, waves
    split K), the tiled kernels otherwise — the same fused epilogue (bias, LoRA K-ext, gelu,
    pre-activation, residual) vs the fp32 reference, and equal to the tiled kernel (tile 4) within
    accumulation-order rounding."""
    C = _C()
    torch.manual_seed(3)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    a2 = torch.randn(M, 32, device="cuda", dtype=torch.bfloat16)
    b2 = torch.randn(N, 32, device="cuda", dtype=torch.bfloat16) * 0.1
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    out, pre = _gnt(C, a, b, bias, a2, b2, 1, None, res, 0.0, 0, True, 1.0, None, 0, None, None, 0.0, 0)
    exp, exp_pre = ref.gemm_nt(a, b, bias, a2, b2, 1, None, res, 0.0, 0, True)
    torch.testing.assert_close(pre.float(), exp_pre.float(), atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(out.float(), exp.float(), atol=8e-2, rtol=3e-2)
    tiled = _gnt(C, a, b, bias, a2, b2, 1, None, res, 0.0, 0, True, 1.0, None, 4, None, None, 0.0, 0)
    torch.testing.assert_close(out.float(), tiled[0].float(), atol=3e-2, rtol=2e-2)
    plain = C.gemm_nt(a, b, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0,
                      None, 32, 0.0, 0)[0]
    torch.testing.assert_close(plain.float(), a.float() @ b.float().t(), atol=3e-2, rtol=2e-2)
    again = _gnt(C, a, b, bias, a2, b2, 1, None, res, 0.0, 0, True, 1.0, None, 0, None, None, 0.0, 0)[0]
    assert torch.equal(out, again)  # deterministic


@pytest.mark.parametrize("rows", [8, 24])
@pytest.mark.parametrize("K", [768, 3072])
def test_gemm_skinny_epilogue_projection(rows, K):
    """The skinny kernel's next-adapter projection slabs == lora_proj over its stored output (K = 3072:
    the K-split form, whose last-arriving block runs the epilogue and the projection)."""
    C = _C()
    torch.manual_seed(9)
    M, N = 64, 3072
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    bias = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    pw = torch.zeros(32, N, device="cuda", dtype=torch.bfloat16)
    pw[:rows] = (0.05 * torch.randn(rows, N, device="cuda")).to(torch.bfloat16)
    out, pre, t = C.gemm_nt(a, b, bias, None, None, 1, None, None, 0.0, 0, True, 1.0, None, 0, None, None, 0.0, 0,
                            pw, rows, 0.0, 4321)
    exp = C.lora_proj(out, pw, 1.0, 0.0, 4321, rows)
    torch.testing.assert_close(t.float(), exp.float(), atol=2e-2, rtol=1e-2)
    assert float(t[:, rows if rows > 16 else 16:].abs().max()) == 0.0


def test_decode_tail_matches_torch():
    """decode_tail == the torch ops it replaces: argmax (first maximal index, ties, -inf rows),
    pad for finished rows, out[b, col[b]], done |= eos, next ids, col / pos / t advance."""
    from mift.ops import kernels as K
    torch.manual_seed(2)
    B, V, Vp, max_new, fill, pad, eos = 64, 50257, 50304, 16, 7, 50256, 11
    full = torch.randn(B, Vp, device="cuda").to(torch.bfloat16)
    full[3, 100] = full[3, 200] = 50.0  # tie: first index wins
    full[5, :V] = float("-inf")  # all -inf: index 0
    full[6, 11] = 60.0  # emits eos
    full[:, V:] = 99.0  # padding columns are never candidates
    logits = full[:, :V]
    done = torch.zeros(B, dtype=torch.bool, device="cuda")
    done[9] = True
    ids = torch.zeros(B, 1, dtype=torch.long, device="cuda")
    out = torch.zeros(B, max_new, dtype=torch.long, device="cuda")
    col = torch.full((B, 1), 4, dtype=torch.long, device="cuda")
    pos = torch.arange(B, device="cuda")[:, None].clone()
    t = torch.tensor([33], dtype=torch.int32, device="cuda")
    d0 = done.clone()
    K.decode_tail(logits, V, done, ids, out, col, pos, t, fill, pad, eos)
    nx = logits.float().argmax(-1)
    assert int(nx[3]) == 100 and int(nx[5]) == 0
    nx = torch.where(d0, torch.full_like(nx, pad), nx)
    assert torch.equal(out[:, 4], nx) and int(out[:, :4].abs().sum()) == 0
    dn = d0 | (nx == eos)
    assert torch.equal(done, dn) and bool(done[6]) and bool(done[9])
    assert torch.equal(ids[:, 0], torch.where(dn, torch.full_like(nx, fill), nx))
    assert int(col.min()) == 5 and int(col.max()) == 5
    assert torch.equal(pos[:, 0], torch.arange(B, device="cuda") + 1) and int(t) == 34


@pytest.mark.parametrize("M", [1, 13, 64])
@pytest.mark.parametrize("N,K,act", [(2304, 768, 0), (3072, 768, 1), (1024, 1024, 2)])
def test_gemm_ln_prologue(M, N, K, act):
    """gemm_ln (decode): act(LayerNorm(x) @ w.T + bias) in one launch == layer_norm_fwd + gemm_nt."""
    from mift.ops import kernels as K_
    torch.manual_seed(4)
    x = (torch.randn(M, K, device="cuda") * 3 + 1).to(torch.bfloat16)
    lw = (1 + 0.1 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    lb = (0.1 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    bias = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    assert K_.gemm_ln_ok(x, w, lw)
    y = K_.gemm_ln(x, lw, lb, 1e-5, w, bias, act=act)
    a, _, _ = K_.layer_norm_fwd(x, lw, lb, 1e-5)
    exp = K_.gemm(a, w, bias, act=act, tile=4)
    # the in-GEMM statistics sum in another order: single LN outputs may round to the neighbouring
    # 16-bit value, and a handful of such flips moves an output by a few 1e-2
    torch.testing.assert_close(y.float(), exp.float(), atol=6e-2, rtol=2e-2)
    ref_a = torch.nn.functional.layer_norm(x.float(), (K,), lw.float(), lb.float(), 1e-5)
    z = ref_a @ w.float().t() + bias.float()
    ref_y = {0: z, 1: torch.nn.functional.gelu(z, approximate="tanh"), 2: torch.relu(z)}[act]
    torch.testing.assert_close(y.float(), ref_y, atol=6e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [1, 13, 64])
@pytest.mark.parametrize("N,K,act,dt", [(2304, 768, 0, torch.bfloat16), (3072, 768, 1, torch.bfloat16),
                                        (1024, 1024, 2, torch.float16), (768, 768, 0, torch.float16)])
def test_gemm_ln_fold(M, N, K, act, dt):
    """gemm_ln_fold (decode, LN folded into the weights: rstd·(x·(γ∘w)ᵀ − mean·c1) + c2) against the fp32
    reference of act(LayerNorm(x) @ w.T + bias), at GPT-2-like residual rows (mean offset, one outlier
    column), and against the LN-prologue form; the fold cache is rebuilt after an in-place update."""
    from mift.ops import fused as F
    from mift.ops import kernels as K_
    torch.manual_seed(5)
    x = torch.randn(M, K, device="cuda") * 3 + 1
    x[:, 7] = 40.0  # an outlier dimension as in GPT-2's residual stream
    x = x.to(dt)
    ln = torch.nn.LayerNorm(K, eps=1e-5, device="cuda", dtype=dt)
    with torch.no_grad():
        ln.weight.copy_(1 + 0.1 * torch.randn(K, device="cuda"))
        ln.bias.copy_(0.1 * torch.randn(K, device="cuda"))

    class Lin:
        pass

    lin = Lin()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
    lin.bias = (0.1 * torch.randn(N, device="cuda")).to(dt)
    y = F._gemm_ln(x, ln, lin, w, act=act)
    ref_a = torch.nn.functional.layer_norm(x.float(), (K,), ln.weight.float(), ln.bias.float(), 1e-5)
    z = ref_a @ w.float().t() + lin.bias.float()
    ref_y = {0: z, 1: torch.nn.functional.gelu(z, approximate="tanh"), 2: torch.relu(z)}[act]
    torch.testing.assert_close(y.float(), ref_y, atol=6e-2, rtol=3e-2)
    y1 = K_.gemm_ln(x, ln.weight, ln.bias, 1e-5, w, lin.bias, act=act)
    torch.testing.assert_close(y.float(), y1.float(), atol=8e-2, rtol=3e-2)
    with torch.no_grad():
        ln.weight.mul_(2.0)  # in place: version counter bumps, the folded operands must follow
    y2 = F._gemm_ln(x, ln, lin, w, act=act)
    ref_a2 = torch.nn.functional.layer_norm(x.float(), (K,), ln.weight.float(), ln.bias.float(), 1e-5)
    z2 = ref_a2 @ w.float().t() + lin.bias.float()
    ref_y2 = {0: z2, 1: torch.nn.functional.gelu(z2, approximate="tanh"), 2: torch.relu(z2)}[act]
    torch.testing.assert_close(y2.float(), ref_y2, atol=1e-1, rtol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("D,rank,p,dres,wf32,dt", [(768, 8, 0.1, True, False, torch.bfloat16),
                                                  (768, 24, 0.0, True, False, torch.bfloat16),
                                                  (1024, 8, 0.1, False, True, torch.bfloat16),
                                                  (768, 8, 0.1, True, True, torch.bfloat16),
                                                  (2560, 24, 0.1, True, False, torch.float16),
                                                  (2560, 8, 0.0, False, True, torch.float16),
                                                  (2048, 8, 0.1, True, False, torch.bfloat16),
                                                  (2560, 8, 0.1, True, True, torch.bfloat16)])
def test_ln_bwd_mask_proj_matches_separate_passes(D, rank, p, dres, wf32, dt):
    """rowproj MODE 3 (LN backward + residual-dropout backward + dT projection in one pass) against
    layer_norm_bwd followed by mask_proj, and against the fp32 reference of the three ops (the OPT
    widths run the 8- and 16-wave forms)."""
    from mift.ops import kernels as K
    torch.manual_seed(3)
    M = 1000
    x = torch.randn(M, D, device="cuda").to(dt)
    dy = torch.randn(M, D, device="cuda").to(dt)
    w = (1 + 0.1 * torch.randn(D, device="cuda")).to(torch.float32 if wf32 else dt)
    b = torch.zeros(D, device="cuda", dtype=w.dtype)
    _, mean, rstd = K.layer_norm_fwd(x, w, b, 1e-5)
    gr = torch.randn(M, D, device="cuda").to(dt) if dres else None
    pw = torch.zeros(32, D, device="cuda", dtype=dt)
    pw[:rank] = (torch.randn(rank, D, device="cuda") / D ** 0.5).to(dt)
    dh, y, pr = K.ln_bwd_mask_proj(dy, x, w, mean, rstd, gr, p, 77, pw, rank, 0.5)
    dh0 = K.layer_norm_bwd(dy, x, w, mean, rstd, dres=gr)[0]
    y0, pr0 = K.mask_proj(dh0, p, 77, pw, rank, 0.5)
    # the row sums run in another order: dh within one 16-bit rounding of the separate pass
    torch.testing.assert_close(dh.float(), dh0.float(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(y.float(), y0.float(), atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(pr.float(), pr0.float(), atol=3e-2, rtol=2e-2)
    if p == 0:
        assert y.data_ptr() == dh.data_ptr()
    # fp32 reference of LN backward + residual
    xf = x.float().requires_grad_(True)
    yf = torch.nn.functional.layer_norm(xf, (D,), w.float(), b.float(), 1e-5)
    yf.backward(dy.float())
    ref = xf.grad + (gr.float() if dres else 0)
    torch.testing.assert_close(dh.float(), ref, atol=3e-2, rtol=2e-2)
    keep = (y0 != 0) | (dh0 == 0)
    torch.testing.assert_close((pr.float()[:, :rank]), (0.5 * y.float() @ pw.float()[:rank].t()), atol=3e-2, rtol=2e-2)
    assert keep.all() if p == 0 else True


@pytest.mark.parametrize("S", [7, 256, 700])
def test_mask_positions_matches_torch(S):
    """mask_positions (one launch) == HF-style cumsum(mask)·mask - 1 and Σ mask, for right-, left- and
    middle-padded int64 masks, S below / at / above one 256-token chunk."""
    from mift.models.opt import opt_positions
    from mift.ops import kernels as K_
    torch.manual_seed(1)
    B = 9
    mask = torch.ones(B, S, dtype=torch.int64, device="cuda")
    for b in range(B):
        n = int(torch.randint(0, S + 1, (1,)))
        if b % 3 == 0:
            mask[b, n:] = 0       # right padding
        elif b % 3 == 1:
            mask[b, :S - n] = 0   # left padding
        else:
            mask[b] = (torch.rand(S, device="cuda") > 0.3).long()
    pos, kv = K_.mask_positions(mask)
    assert torch.equal(pos, opt_positions(mask))
    assert torch.equal(kv, mask.sum(1, dtype=torch.int32))


@pytest.mark.parametrize("tile", [7, 8, 9, 10])
@pytest.mark.parametrize("epi", ["fwd", "dgrad_masked"])
def test_gemm_hoisted_dropout_hash_bit_identical(tile, epi, monkeypatch):
    """The epilogues' dropout-mask hashes from the hoisted high-word mix (MIFT_EPI_HOIST=1, default:
    residual-dropout keep8 in the staged phase 2, masked K-extension keep4 in phase 1) draw exactly the
    masks of the per-call form (MIFT_EPI_HOIST=0)."""
    C = _C()
    torch.manual_seed(9)
    M, N, K = 1536, 3072 if tile == 9 else 2304, 768
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    a2 = torch.randn(M, 32, device="cuda", dtype=torch.bfloat16)
    b2 = torch.randn(N, 32, device="cuda", dtype=torch.bfloat16) * 0.1
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    outs = []
    for h in ("0", "1"):
        monkeypatch.setenv("MIFT_EPI_HOIST", h)
        if epi == "fwd":
            outs.append(_gnt(C, a, b, bias, a2, b2, 0, None, res, 0.1, 5, False, 1.0, None, tile, None, None, 0.0, 0)[0])
        else:
            outs.append(_gnt(C, a, b, None, a2, b2, 4, aux, None, 0.0, 0, False, 1.0, None, tile, None, None, 0.05, 77)[0])
    assert torch.equal(outs[0], outs[1])
