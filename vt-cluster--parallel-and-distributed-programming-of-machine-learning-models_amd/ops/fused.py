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
    """Per-forward packed 16-bit LoRA operands of one Linear."""
    __slots__ = ("A32", "B32", "r", "s", "p")

    def __init__(self, lin, dtype):
        A, B = lin.lora_A.weight, lin.lora_B.weight
        self.r, self.s, self.p = lin.lora_r, lin.lora_scaling, lin.lora_dropout
        self.A32, self.B32 = K.pack_lora(A.detach(), B.detach(), self.s, dtype)  # A32 pre-scaled by s


def _lora_fwd(x, lo: "LoraOperands", seed, training):
    """Returns (xd, T32): xd = dropout(x) (or x), T32 = xd @ (s A)^T padded to 32 cols."""
    if training and lo.p > 0:
        xd = K.mask_scale(x, lo.p, seed)
    else:
        xd = x
    T32 = K.gemm(xd, lo.A32)
    return xd, T32


def _lora_bwd(gz, xd, T32, lo: "LoraOperands", dx, seed, training):
    """LoRA grads from gz = dL/d(pre-activation output). Adds input grad into dx."""
    r = lo.r
    dB = (gz.t() @ T32[:, :r]).float()                     # [N, r]
    dT = gz @ lo.B32[:, :r]                                  # [M, r]
    dA = (dT.t() @ xd).float() * lo.s                        # [r, K]
    dxd = dT @ lo.A32[:r]                                    # [M, K] (A32 carries s)
    if training and lo.p > 0:
        K.mask_scale(dxd, lo.p, seed, out=dx, accumulate=True)
    else:
        dx.add_(dxd)
    return dA, dB


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
        xd = T32 = None
        if lo is not None:
            xd, T32 = _lora_fwd(a, lo, lora_seed, training)
        y = K.gemm(a, lin.w_nk(), lin.bias, T32, lo.B32 if lo else None)
        ctx.save_for_backward(x2, a, mean, rstd, ln_w, xd if (lo and xd is not a) else None, T32)
        ctx.lin, ctx.lo, ctx.eps, ctx.seed, ctx.training, ctx.shp = lin, lo, eps, lora_seed, training, shp
        return y.view(*shp[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, gy):
        x2, a, mean, rstd, ln_w, xd, T32 = ctx.saved_tensors
        lin, lo = ctx.lin, ctx.lo
        gy = _flat(gy.contiguous())
        da = K.gemm(gy, lin.w_kn())
        dA = dB = None
        if lo is not None:
            dA, dB = _lora_bwd(gy, xd if xd is not None else a, T32, lo, da, ctx.seed, ctx.training)
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
        xd = T32 = None
        if lo is not None:
            xd, T32 = _lora_fwd(x2, lo, lora_seed, training)
        pp = p if training else 0.0
        y = K.gemm(x2, lin.w_nk(), lin.bias, T32, lo.B32 if lo else None, residual=h2, dropout_p=pp, seed=seed)
        ctx.save_for_backward(x2, xd if (lo and xd is not x2) else None, T32)
        ctx.lin, ctx.lo, ctx.p, ctx.seed, ctx.lseed, ctx.training, ctx.xshp = lin, lo, pp, seed, lora_seed, training, x.shape
        return y.view(shp)

    @staticmethod
    def backward(ctx, gh):
        x2, xd, T32 = ctx.saved_tensors
        lin, lo = ctx.lin, ctx.lo
        gh2 = _flat(gh.contiguous())
        gz = K.mask_scale(gh2, ctx.p, ctx.seed) if ctx.p > 0 else gh2
        dx = K.gemm(gz, lin.w_kn())
        dA = dB = None
        if lo is not None:
            dA, dB = _lora_bwd(gz, xd if xd is not None else x2, T32, lo, dx, ctx.lseed, ctx.training)
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
        ad = T1 = fd = T2 = None
        if lo1 is not None:
            ad, T1 = _lora_fwd(a, lo1, seed_l1, training)
        f, z = K.gemm(a, fc1.w_nk(), fc1.bias, T1, lo1.B32 if lo1 else None, act=act, want_preact=True)
        if lo2 is not None:
            fd, T2 = _lora_fwd(f, lo2, seed_l2, training)
        pp = p if training else 0.0
        out = K.gemm(f, fc2.w_nk(), fc2.bias, T2, lo2.B32 if lo2 else None, residual=h2, dropout_p=pp, seed=seed)
        ctx.save_for_backward(h2, a, mean, rstd, ln_w, z, f,
                              ad if (lo1 and ad is not a) else None, T1,
                              fd if (lo2 and fd is not f) else None, T2)
        ctx.fc1, ctx.fc2, ctx.lo1, ctx.lo2 = fc1, fc2, lo1, lo2
        ctx.act, ctx.p, ctx.seed, ctx.sl1, ctx.sl2, ctx.training, ctx.shp = act, pp, seed, seed_l1, seed_l2, training, shp
        return out.view(shp)

    @staticmethod
    def backward(ctx, gh):
        h2, a, mean, rstd, ln_w, z, f, ad, T1, fd, T2 = ctx.saved_tensors
        fc1, fc2, lo1, lo2 = ctx.fc1, ctx.fc2, ctx.lo1, ctx.lo2
        gh2 = _flat(gh.contiguous())
        gm = K.mask_scale(gh2, ctx.p, ctx.seed) if ctx.p > 0 else gh2
        dA1 = dB1 = dA2 = dB2 = None
        if lo2 is None:
            # dZ = (gm @ W2) * act'(z) fused in the dgrad epilogue
            dz = K.gemm(gm, fc2.w_kn(), act=_BWD[ctx.act], aux=z)
        else:
            df = K.gemm(gm, fc2.w_kn())
            dA2, dB2 = _lora_bwd(gm, fd if fd is not None else f, T2, lo2, df, ctx.sl2, ctx.training)
            dz = K.act_bwd(df, z, ctx.act)
        da = K.gemm(dz, fc1.w_kn())
        if lo1 is not None:
            dA1, dB1 = _lora_bwd(dz, ad if ad is not None else a, T1, lo1, da, ctx.sl1, ctx.training)
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
        logits = K.gemm(a, w_nk)
        loss_rows, _ = K.xent(logits, labels.reshape(-1), V, ignore_index, write_grad=need_grad)
        if need_grad:
            ctx.save_for_backward(h2, mean, rstd, ln_w, logits, w_kn)
        ctx.eps, ctx.shp = eps, shp
        return loss_rows.sum()

    @staticmethod
    def backward(ctx, g):
        h2, mean, rstd, ln_w, dlogits, w_kn = ctx.saved_tensors
        g = g.reshape(1).float().contiguous()
        da = K.gemm(dlogits, w_kn, alpha_t=g)
        dh, _, _, _ = K.layer_norm_bwd(da, h2, ln_w, mean, rstd)
        return dh.view(ctx.shp), None, None, None, None, None, None, None, None, None


def lm_head_xent(h, ln, w_nk, w_kn, labels, V, ignore_index=-100, need_grad=True):
    return LMHeadXent.apply(h, ln.weight, ln.bias, ln.eps, w_nk, w_kn, labels, V, ignore_index, need_grad)


def lm_head_logits(h, ln, w_nk, V):
    h2 = _flat(h.contiguous())
    a, _, _ = K.layer_norm_fwd(h2, ln.weight, ln.bias, ln.eps)
    logits = K.gemm(a, w_nk)
    return logits[:, :V].view(*h.shape[:-1], V)
