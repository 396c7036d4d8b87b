"""Block-level fused autograd Functions over the gfx950 kernels.

Each Function owns a whole sub-graph of a transformer block and writes its
own backward, so fusions can cross what would be op boundaries in eager
PyTorch:

* ``ln_linear``      y = LoRALinear(LN(x))                       (qkv projection)
* ``linear_residual`` h' = h + dropout(LoRALinear(x))            (attention out-proj)
* ``mlp``            h' = h + dropout(fc2(act(fc1(LN(h)))))      (LoRA on either fc)
* ``lm_head_xent``   sum CE(LN(h) @ E^T, labels)                 (tied head + loss)

LoRA inside a GEMM: T = s·dropout(X)·A^T is computed into a [M,32] bf16
panel and fed to the base GEMM as a K-extension (one extra MFMA K-step, see
csrc/kernels/gemm.hip), so the adapter never needs its own output pass.
Backward: dX from the frozen W^T copy (MFMA GEMM, activation-backward fused
in its epilogue where the producer allows), LoRA grads dA/dB from the
rank-r panels (skinny products), LoRA input-dropout mask regenerated from
its counter seed.
"""
import torch

from . import kernels as K

_BWD = {0: 0, 1: 4, 2: 5, 3: 6}


class LoraOperands:
    """Per-forward packed 16-bit LoRA operands of one Linear (rank padded to 32).

    A32s [32,K] = s·A (forward projection), B32 [N,32] (forward K-extension),
    B32t [32,N] = B^T (backward dT = s·gz·B), At32 [K,32] = A^T (dgrad K-extension)."""
    __slots__ = ("A32s", "B32", "B32t", "At32", "r", "s", "p", "arena", "offA", "offB", "K", "N")

    def __init__(self, lin, dtype):
        self.r, self.s, self.p = lin.lora_r, lin.lora_scaling, lin.lora_dropout
        self.K, self.N = lin.in_features, lin.out_features
        pk = getattr(lin, "_pack_owner", None)
        self.arena = getattr(lin, "_arena", None)
        if self.arena is not None:
            self.offA, self.offB = lin._offA, lin._offB
        if pk is not None and pk.dtype == dtype:
            pk.refresh()
            self.A32s, self.B32, self.B32t, self.At32 = lin._pack
            return
        A, B = lin.lora_A.weight.detach(), lin.lora_B.weight.detach()
        self.A32s, self.B32 = K.pack_lora(A, B, self.s, dtype)
        r = self.r
        self.B32t = torch.zeros(32, B.shape[0], dtype=dtype, device=B.device)
        self.B32t[:r].copy_(B.t())
        self.At32 = torch.zeros(A.shape[1], 32, dtype=dtype, device=A.device)
        self.At32[:, :r].copy_(A.t())


def _lora_fwd(x, lo: "LoraOperands", seed, training):
    """T32 = s·dropout(x)·A^T  [M,32] (mask applied in-register, x_drop never stored)."""
    p = lo.p if training else 0.0
    return K.lora_proj(x, lo.A32s, 1.0, p, seed)


def _lora_bwd(gz, x, T32, lo: "LoraOperands", seed, training):
    """LoRA grads from gz = dL/d(pre-activation output).

    Returns (dA [r,K], dB [N,r], dT32) where dT32 = s·gz·B feeds the dgrad
    GEMM's masked K-extension (dX += keep ⊙ dT32·A^T / (1-p))."""
    r = lo.r
    p = lo.p if training else 0.0
    dT32 = K.lora_proj(gz, lo.B32t, lo.s, 0.0, 0)                 # s·gz·B        [M,32]
    if lo.arena is not None:
        # accumulate straight into the flat fp32 grad arena (no temporaries,
        # no autograd accumulation pass); autograd sees None for A/B
        g = lo.arena.grad
        K.lora_wgrad_into(gz, T32, g, 1, r, lo.offB)               # dB [N,r]
        K.lora_wgrad_into(x, dT32, g, 2, r, lo.offA, p, seed)      # dA [r,K]
        return None, None, dT32
    dBf = K.lora_wgrad(gz, T32)                                   # gz^T·T        [N,32]
    dAf = K.lora_wgrad(x, dT32, p=p, seed=seed)                   # drop(x)^T·s·dT [K,32]
    return dAf[:, :r].t(), dBf[:, :r], dT32


def _dgrad(gz, lin, lo, dT32, seed, training, **kw):
    """dX = gz·W (+ masked LoRA K-extension)."""
    if lo is None:
        return K.gemm(gz, lin.w_kn(), **kw)
    p = lo.p if training else 0.0
    return K.gemm(gz, lin.w_kn(), a2=dT32, b2=lo.At32, ext_p=p, ext_seed=seed, **kw)


def _flat(x):
    return x.reshape(-1, x.shape[-1])


# ---------------------------------------------------------------------------
class LnLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ln_w, ln_b, A, B, lin, eps, lora_seed, training):
        shp = x.shape
        x2 = _flat(x.contiguous())
        a, mean, rstd = K.layer_norm_fwd(x2, ln_w, ln_b, eps)
        lo = LoraOperands(lin, x.dtype) if lin.lora_r > 0 else None
        T32 = _lora_fwd(a, lo, lora_seed, training) if lo is not None else None
        y = K.gemm(a, lin.w_nk(), lin.bias, T32, lo.B32 if lo else None)
        ctx.save_for_backward(x2, a, mean, rstd, ln_w, T32)
        ctx.lin, ctx.lo, ctx.eps, ctx.seed, ctx.training, ctx.shp = lin, lo, eps, lora_seed, training, shp
        return y.view(*shp[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, gy):
        x2, a, mean, rstd, ln_w, T32 = ctx.saved_tensors
        lin, lo = ctx.lin, ctx.lo
        gy = _flat(gy.contiguous())
        dA = dB = dT32 = None
        if lo is not None:
            dA, dB, dT32 = _lora_bwd(gy, a, T32, lo, ctx.seed, ctx.training)
        da = _dgrad(gy, lin, lo, dT32, ctx.seed, ctx.training)
        dx, _, _, _ = K.layer_norm_bwd(da, x2, ln_w, mean, rstd)
        return dx.view(ctx.shp), None, None, dA, dB, None, None, None, None


def ln_linear(x, ln, lin, lora_seed=0, training=True):
    A = lin.lora_A.weight if lin.lora_r > 0 else None
    B = lin.lora_B.weight if lin.lora_r > 0 else None
    return LnLinear.apply(x, ln.weight, ln.bias, A, B, lin, ln.eps, lora_seed, training)


# ---------------------------------------------------------------------------
class LinearResidual(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h, A, B, lin, p, seed, lora_seed, training):
        shp = h.shape
        x2 = _flat(x.contiguous())
        h2 = _flat(h.contiguous())
        lo = LoraOperands(lin, x.dtype) if lin.lora_r > 0 else None
        T32 = _lora_fwd(x2, lo, lora_seed, training) if lo is not None else None
        pp = p if training else 0.0
        y = K.gemm(x2, lin.w_nk(), lin.bias, T32, lo.B32 if lo else None, residual=h2, dropout_p=pp, seed=seed)
        ctx.save_for_backward(x2, T32)
        ctx.lin, ctx.lo, ctx.p, ctx.seed, ctx.lseed, ctx.training, ctx.xshp = lin, lo, pp, seed, lora_seed, training, x.shape
        return y.view(shp)

    @staticmethod
    def backward(ctx, gh):
        x2, T32 = ctx.saved_tensors
        lin, lo = ctx.lin, ctx.lo
        gh2 = _flat(gh.contiguous())
        gz = K.mask_scale(gh2, ctx.p, ctx.seed) if ctx.p > 0 else gh2
        dA = dB = dT32 = None
        if lo is not None:
            dA, dB, dT32 = _lora_bwd(gz, x2, T32, lo, ctx.lseed, ctx.training)
        dx = _dgrad(gz, lin, lo, dT32, ctx.lseed, ctx.training)
        return dx.view(ctx.xshp), gh, dA, dB, None, None, None, None, None


def linear_residual(x, h, lin, p, seed, lora_seed=0, training=True):
    A = lin.lora_A.weight if lin.lora_r > 0 else None
    B = lin.lora_B.weight if lin.lora_r > 0 else None
    return LinearResidual.apply(x, h, A, B, lin, p, seed, lora_seed, training)


# ---------------------------------------------------------------------------
class MLP(torch.autograd.Function):
    """h' = h + dropout(fc2(act(fc1(LN(h)))))."""

    @staticmethod
    def forward(ctx, h, ln_w, ln_b, A1, B1, A2, B2, fc1, fc2, eps, act, p, seed, seed_l1, seed_l2, training):
        shp = h.shape
        h2 = _flat(h.contiguous())
        a, mean, rstd = K.layer_norm_fwd(h2, ln_w, ln_b, eps)
        lo1 = LoraOperands(fc1, h.dtype) if fc1.lora_r > 0 else None
        lo2 = LoraOperands(fc2, h.dtype) if fc2.lora_r > 0 else None
        T1 = _lora_fwd(a, lo1, seed_l1, training) if lo1 is not None else None
        f, z = K.gemm(a, fc1.w_nk(), fc1.bias, T1, lo1.B32 if lo1 else None, act=act, want_preact=True)
        T2 = _lora_fwd(f, lo2, seed_l2, training) if lo2 is not None else None
        pp = p if training else 0.0
        out = K.gemm(f, fc2.w_nk(), fc2.bias, T2, lo2.B32 if lo2 else None, residual=h2, dropout_p=pp, seed=seed)
        ctx.save_for_backward(h2, a, mean, rstd, ln_w, z, f, T1, T2)
        ctx.fc1, ctx.fc2, ctx.lo1, ctx.lo2 = fc1, fc2, lo1, lo2
        ctx.act, ctx.p, ctx.seed, ctx.sl1, ctx.sl2, ctx.training, ctx.shp = act, pp, seed, seed_l1, seed_l2, training, shp
        return out.view(shp)

    @staticmethod
    def backward(ctx, gh):
        h2, a, mean, rstd, ln_w, z, f, T1, T2 = ctx.saved_tensors
        fc1, fc2, lo1, lo2 = ctx.fc1, ctx.fc2, ctx.lo1, ctx.lo2
        gh2 = _flat(gh.contiguous())
        gm = K.mask_scale(gh2, ctx.p, ctx.seed) if ctx.p > 0 else gh2
        dA1 = dB1 = dA2 = dB2 = dT2 = dT1 = None
        if lo2 is not None:
            dA2, dB2, dT2 = _lora_bwd(gm, f, T2, lo2, ctx.sl2, ctx.training)
        # dZ = (gm·W2 [+ masked LoRA ext]) ⊙ act'(z), all in the dgrad epilogue
        dz = _dgrad(gm, fc2, lo2, dT2, ctx.sl2, ctx.training, act=_BWD[ctx.act], aux=z)
        if lo1 is not None:
            dA1, dB1, dT1 = _lora_bwd(dz, a, T1, lo1, ctx.sl1, ctx.training)
        da = _dgrad(dz, fc1, lo1, dT1, ctx.sl1, ctx.training)
        dh, _, _, _ = K.layer_norm_bwd(da, h2, ln_w, mean, rstd, dres=gh2)
        return (dh.view(ctx.shp), None, None, dA1, dB1, dA2, dB2) + (None,) * 9


def mlp(h, ln, fc1, fc2, act, p, seed, seed_l1=0, seed_l2=0, training=True):
    A1 = fc1.lora_A.weight if fc1.lora_r > 0 else None
    B1 = fc1.lora_B.weight if fc1.lora_r > 0 else None
    A2 = fc2.lora_A.weight if fc2.lora_r > 0 else None
    B2 = fc2.lora_B.weight if fc2.lora_r > 0 else None
    return MLP.apply(h, ln.weight, ln.bias, A1, B1, A2, B2, fc1, fc2, ln.eps, act, p, seed, seed_l1, seed_l2,
                     training)


# ---------------------------------------------------------------------------
class LMHeadXent(torch.autograd.Function):
    """Sum of token CE of LN(h) @ E^T against (already shifted) labels.

    Forward computes logits into a [M, V_pad] buffer and turns it into
    dlogits in place (xent kernel); backward is one dgrad GEMM whose
    device-side alpha is the upstream gradient (loss scale / token count)."""

    @staticmethod
    def forward(ctx, h, ln_w, ln_b, eps, w_nk, w_kn, labels, V, ignore_index, need_grad):
        shp = h.shape
        h2 = _flat(h.contiguous())
        a, mean, rstd = K.layer_norm_fwd(h2, ln_w, ln_b, eps)
        # plain library GEMM (no epilogue to fuse): hipBLASLt wins at 8192x50304x768
        logits = torch.matmul(a, w_nk.t())
        loss_rows, _ = K.xent(logits, labels.reshape(-1), V, ignore_index, write_grad=need_grad)
        if need_grad:
            ctx.save_for_backward(h2, mean, rstd, ln_w, logits, w_kn)
        ctx.eps, ctx.shp, ctx.w_nk = eps, shp, w_nk
        return loss_rows.sum()

    @staticmethod
    def backward(ctx, g):
        h2, mean, rstd, ln_w, dlogits, w_kn = ctx.saved_tensors
        g = g.reshape(1).float().contiguous()
        da = torch.matmul(dlogits, ctx.w_nk).mul_(g.to(dlogits.dtype))
        dh, _, _, _ = K.layer_norm_bwd(da, h2, ln_w, mean, rstd)
        return dh.view(ctx.shp), None, None, None, None, None, None, None, None, None


def lm_head_xent(h, ln, w_nk, w_kn, labels, V, ignore_index=-100, need_grad=True):
    return LMHeadXent.apply(h, ln.weight, ln.bias, ln.eps, w_nk, w_kn, labels, V, ignore_index, need_grad)


def lm_head_logits(h, ln, w_nk, V):
    h2 = _flat(h.contiguous())
    a, _, _ = K.layer_norm_fwd(h2, ln.weight, ln.bias, ln.eps)
    logits = K.gemm(a, w_nk)
    return logits[:, :V].view(*h.shape[:-1], V)
