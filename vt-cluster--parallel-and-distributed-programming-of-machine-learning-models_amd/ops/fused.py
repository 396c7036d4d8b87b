"""Block-level fused autograd Functions over the gfx950 kernels.

Each Function owns a whole sub-graph of a transformer block and writes its
own backward, so fusions can cross what would be op boundaries in eager
PyTorch:

* ``ln_linear``       y = LoRALinear(LN(x))                       (qkv projection)
* ``linear_residual`` h' = h + dropout(LoRALinear(x))             (attention out-proj)
* ``mlp``             h' = h + dropout(fc2(act(fc1(LN(h)))))      (LoRA on either fc)
* ``lm_head_xent``    sum CE(LN(h) @ E^T, labels)                 (tied head + loss)

LoRA inside a GEMM: T = s·dropout(X)·A^T is computed into a [M,32] 16-bit
panel (``lora_proj``) and fed to the base GEMM as a K-extension (one extra
MFMA K-step, csrc/kernels/gemm.hip), so the adapter never needs its own
output pass.  Backward: dT = s·gz·B (``lora_proj``), dB/dA by the split-M
transpose-read MFMA kernel (``lora_wgrad``) accumulated straight into the
flat fp32 grad arena, and dX = gz·W^T + keep ⊙ dT·A^T as ONE GEMM whose
K-extension is masked in the epilogue.  The LoRA-input dropout mask is never
stored: every consumer regenerates it from its counter seed.

Any projection object passed as ``lin`` provides ``w_nk()``, ``w_kn()``,
``bias``, ``lora_params()`` and ``lora_ops(dtype)``; the latter returns an
adapter-operand object (``AdapterOps`` for one adapter, or the multi-adapter
variant used by OPT's fused q/k/v projection — mift.models.opt).
"""
import os

import torch

from . import kernels as K
from .streams import join as join_side, run_side

# The fused row passes (LN / dropout-bwd / LN-bwd + the LoRA projection, csrc/kernels/rowproj.hip) run
# their MFMA 16-row form at the widths below (4 waves per block at 768 / 1024, 8 at 2048 / 2560, 16 at
# 4096: OPT-125m .. 6.7b), per pass where it measured no slower than the separate passes it replaces
# (tools/bench_rowproj_opt.py at M = 6144, fp16; profiles/r5/bench_rowproj_opt.json): the LN forward +
# projection not at 4096 (42.4 vs 40.8 us), the LN backward + dropout backward + dT not at 4096 (the
# 16-wave form spills: 155 vs 81 us).  Elsewhere only the one-wave-per-row kernels exist, which do LR
# FMAs per element on the VALU with the [LR,D] operand re-read from cache for every row: for OPT's fused
# q/k/v adapters (24 rows -> LR = 32) at D = 2560 they ran 131 us at M = 6144 against 27 for LN + the
# MFMA lora_proj, so there they are limited to few rows and D <= 1024.
_ROWPROJ_D = {"ln": (768, 1024, 2048, 2560), "mask": (768, 1024, 2048, 2560, 4096),
              "ln_bwd": (768, 1024, 2048, 2560)}


def _diag_skip(what):
    """MIFT_DIAG_SKIP=wgrad (diagnostics only, wrong gradients): drop the LoRA weight-grad launches
    to measure their critical-path cost in a whole step (tools/step_ab.py).  Read per call."""
    return what in os.environ.get("MIFT_DIAG_SKIP", "").split(",")

_LNPROJ_MAX_ROWS = int(os.environ.get("MIFT_LNPROJ_MAX_ROWS", "8"))
_LNPROJ_MAX_D = int(os.environ.get("MIFT_LNPROJ_MAX_D", "1024"))


def _mfma_width(D, kind):
    """The MFMA row-pass form runs pass ``kind`` ("ln", "mask", "ln_bwd") at width D
    (MIFT_ROWPROJ_WIDE=0, read per call: only the round-4 widths 768 / 1024 — A/B knob)."""
    return D in (768, 1024) or (D in _ROWPROJ_D[kind] and os.environ.get("MIFT_ROWPROJ_WIDE", "1") != "0")


def _rowproj_fused(D, rows, kind):
    """One fused row pass (LN / dropout-bwd + projection): the MFMA 16-row kernel where _mfma_width
    (any rank), the one-wave-per-row kernel for up to _LNPROJ_MAX_ROWS rows at other D <= 1024."""
    return _mfma_width(D, kind) or (rows <= _LNPROJ_MAX_ROWS and D <= _LNPROJ_MAX_D)


def _ln_fwd_lora(x2, ln_w, ln_b, eps, lo, seed, training):
    """(LN(x), mean, rstd, T32 = s·dropout(LN(x))·Aᵀ) — fused row pass or LN + lora_proj."""
    if _rowproj_fused(x2.shape[-1], lo.rows, "ln"):
        return K.layer_norm_fwd_proj(x2, ln_w, ln_b, eps, lo.A32s, lo.rows, 1.0, lo.p if training else 0.0, seed)
    a, mean, rstd = K.layer_norm_fwd(x2, ln_w, ln_b, eps)
    return a, mean, rstd, lo.forward(a, seed, training)


def _mask_proj(g2, p, seed, lo):
    """(gz = dropout-bwd(g), dT0 = dt_alpha·gz·B) — one row pass where _rowproj_fused (the one-wave-per-row
    form at OPT's D = 2560 ran 79 us against mask_scale + the projection, 38 + 22 us)."""
    if _rowproj_fused(g2.shape[-1], lo.rows, "mask"):
        return K.mask_proj(g2, p, seed, lo.B32t, lo.rows, lo.dt_alpha)
    gz = K.mask_scale(g2, p, seed) if p > 0 else g2
    return gz, K.lora_proj(gz, lo.B32t, lo.dt_alpha, 0.0, 0, rows=lo.rows)

_BWD = {0: 0, 1: 4, 2: 5, 3: 6}


def _epi_proj_kw(lo, seed, training):
    """gemm kwargs that make the producing GEMM's epilogue emit ``lo.forward(out)`` (MIFT_EPI_PROJ=0:
    the separate lora_proj pass, A/B knob read per call)."""
    if lo is None or os.environ.get("MIFT_EPI_PROJ", "1") == "0":
        return {}
    return {"proj_w": lo.A32s, "proj_rows": lo.rows, "proj_p": lo.p if training else 0.0, "proj_seed": seed}


def _epi_dt_kw(lo):
    """gemm kwargs that make a dgrad GEMM's epilogue emit the adapter's backward projection
    dT = dt_alpha·out·Bᵀ of its own output (the gradient entering ``lo``'s linear) — e.g. fc2's dgrad
    producing fc1's dz and its dT in one pass instead of a lora_proj re-reading dz (MIFT_EPI_DT=0, read
    per call: the separate pass)."""
    if lo is None or os.environ.get("MIFT_EPI_DT", "1") == "0":
        return {}
    return {"proj_w": lo.B32t, "proj_rows": lo.rows, "proj_alpha": lo.dt_alpha}


def _claim(arena, offsets):
    """Tell the DP reducer, at forward time, that the fused backward writes these arena grads itself
    and reports them through ``_notify``.  The Functions still take the LoRA tensors as autograd
    inputs (so a block fed by the frozen embedding is still differentiated), and PyTorch runs their
    post-accumulate-grad hooks although the backward returns None for them: counted as well, every
    tensor would be "ready" twice and a bucket's all-reduce would launch before the last layers'
    weight-grad kernels were queued (measured: eager DP2 replicas diverged from step 1,
    tools/diag_ddp_eager.py)."""
    cb = getattr(arena, "grad_claim", None)
    if cb is not None:
        cb(offsets)


def _notify(arena, offsets):
    """Tell the DP reducer (mift.parallel.ddp) that these arena grads are final for this
    micro-step: the wgrad kernels are queued, so its bucket all-reduce can launch now and
    overlap the rest of backward (the fused path never runs AccumulateGrad hooks)."""
    cb = getattr(arena, "grad_ready", None)
    if cb is not None:
        cb(offsets)


class _WgradBatch:
    """LoRA weight-gradient problems deferred to ONE grouped launch (``lora_wgrad_group``).

    The adapters of a transformer layer queue their dB / dA problems here during backward and
    the layer's first Function in forward order (``LnLinear``, i.e. the last one in backward)
    flushes them: one launch per layer instead of two per adapter (each of those paid ~10 us of
    ramp and tail for 12-50 MB of reads).  The inputs stay referenced until the launch, the DP
    reducer is notified after it (bucket all-reduces still overlap the next layer's backward),
    and an end-of-backward callback flushes whatever is left (models without an LnLinear)."""
    MAX = 16

    def __init__(self):
        self.arena = None
        self.xs, self.ys, self.meta, self.ps, self.offs = [], [], [], [], []
        self.cb = False

    def add(self, arena, x, y, mode, slots, p, seed, offs):
        if self.arena is not None and (self.arena is not arena or len(self.xs) >= self.MAX):
            self.flush()
        self.arena = arena
        m = [mode, len(slots)]
        for q, r, o in slots:
            m += [q, r, o]
        m += [0, 0, 0] * (4 - len(slots)) + [seed]
        self.xs.append(x)
        self.ys.append(y)
        self.meta += m
        self.ps.append(p)
        self.offs += list(offs)
        if not self.cb:
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self._final)
                self.cb = True
            except RuntimeError:
                pass  # not inside backward: flushed by the next flush() call

    def reset(self):
        """Drop anything a failed backward left queued (e.g. an OOM after queue_callback): its
        problems must not land in a later step's grads, and the flush callback must re-arm."""
        self.arena = None
        self.xs, self.ys, self.meta, self.ps, self.offs = [], [], [], [], []
        self.cb = False

    def _final(self):
        self.cb = False
        if self.xs:
            self.flush()
            join_side()

    def flush(self):
        if not self.xs:
            return
        arena, xs, ys, meta, ps, offs = self.arena, self.xs, self.ys, self.meta, self.ps, self.offs
        self.arena, self.xs, self.ys, self.meta, self.ps, self.offs = None, [], [], [], [], []
        if not _diag_skip("wgrad"):
            run_side(xs[0].device, lambda: K.lora_wgrad_group(arena.grad, xs, ys, meta, ps), *xs, *ys)
        _notify(arena, offs)


_WG = _WgradBatch()


def flush_wgrads():
    """Launch the queued LoRA weight-gradient problems now (one grouped kernel)."""
    _WG.flush()


def reset_wgrads():
    """Start-of-step hygiene (trainer / graph capture): discard problems a raised backward queued."""
    _WG.reset()


class AdapterOps:
    """Packed 16-bit operands of ONE adapter (rank padded to 32).

    A32s [32,K] = s·A (forward projection), B32 [N,32] (forward K-extension),
    B32t [32,N] = B^T (backward dT = s·gz·B), At32 [K,32] = A^T (dgrad
    K-extension).  Reuses the model's per-optimizer-step pack when present."""

    def __init__(self, lin, dtype):
        self.r, self.s, self.p = lin.lora_r, lin.lora_scaling, lin.lora_dropout
        self.rows, self.dt_alpha = self.r, self.s  # non-zero rows of A32s / B32t; dT = dt_alpha·gz·B32tᵀ
        pk = getattr(lin, "_pack_owner", None)
        self.arena = getattr(lin, "_arena", None)
        if self.arena is not None:
            self.offA, self.offB = lin._offA, lin._offB
            _claim(self.arena, (self.offA, self.offB))
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

    def forward(self, x, seed, training):
        """T32 = s·dropout(x)·A^T  [M,32] (mask applied in-register, never stored)."""
        return K.lora_proj(x, self.A32s, 1.0, self.p if training else 0.0, seed, rows=self.rows)

    def backward(self, gz, x, T32, seed, training, dT32=None):
        """-> (grads for lora_params() [dA, dB] or [None, None], dT32).

        ``dT32`` may come precomputed from the kernel that produced gz (mask_proj)."""
        r = self.r
        p = self.p if training else 0.0
        if dT32 is None:
            dT32 = K.lora_proj(gz, self.B32t, self.s, 0.0, 0, rows=self.rows)  # s·gz·B   [M,32]
        if self.arena is not None:  # dB [N,r] = gzᵀ·T, dA [r,K] = (drop(x)ᵀ·dT)ᵀ, queued for the layer's launch
            _WG.add(self.arena, gz, T32, 1, [(0, r, self.offB)], 0.0, 0, (self.offB,))
            _WG.add(self.arena, x, dT32, 2, [(0, r, self.offA)], p, seed, (self.offA,))
            return [None, None], dT32
        dBf = K.lora_wgrad(gz, T32)
        dAf = K.lora_wgrad(x, dT32, p=p, seed=seed)
        return [dAf[:, :r].t(), dBf[:, :r]], dT32


# Generation of the cached multi-adapter operands: bumped before every hipGraph capture so the
# capture rebuilds them inside the graph (the cache key also holds the arena version, but a capture
# taken right after an eager pass at the SAME version would otherwise bake the eager pass's
# operands in, and every replay would read those stale pre-update values).  ConcatLinear is not an
# nn.Module, so a walk over model.modules() cannot find and clear its cache (the round-3 bug:
# graphed OPT runs drifted from eager from step 2 on).
_PACK_GEN = [0]


def invalidate_packs(model=None):
    """Force every per-step LoRA operand pack to be rebuilt by its next use (call before a capture)."""
    _PACK_GEN[0] += 1
    pk = getattr(model, "_lora_pack", None) if model is not None else None
    if pk is not None:
        pk.version = -1


class MultiAdapterOps:
    """Several adapters on projections that share one input (OPT q/k/v), as
    ONE K-extension: the 32 LoRA columns are split into equal slots, adapter j
    owning columns [w·j, w·j + r_j) with w = 32 // n_adapters.

      A_ext  [32, K]   rows of slot j = s_j·A_j
      B_ext  [N, 32]   block-diagonal: output rows of member j × slot j = B_j
      B_extT [32, N]   s_j·B_j^T in slot j (s baked in: dT = gz·B_extT^T)
      At_ext [K, 32]   A_j^T in slot j

    The LoRA-input dropout mask is generated once per element of the shared
    input, so all adapters of the group see the SAME mask (PEFT draws one per
    adapter; the reference path reproduces the shared mask by passing one
    seed to every member — documented deviation, same distribution).
    Weight grads go slot-by-slot through ``lora_wgrad``'s column offset."""

    def __init__(self, cat, dtype):
        members = [(l, n0, n1) for l, n0, n1 in cat.spans() if l.lora_r > 0]
        self.w = 32 // len(members)
        self.slots = [(l, n0, n1, j * self.w) for j, (l, n0, n1) in enumerate(members)]
        self.rows = max(q + l.lora_r for l, _, _, q in self.slots)
        self.dt_alpha = 1.0  # s_j baked into B_extT
        first = members[0][0]
        self.p = first.lora_dropout
        self.arena = getattr(first, "_arena", None)
        if self.arena is not None:
            _claim(self.arena, [o for l, _, _, _ in self.slots for o in (l._offA, l._offB)])
        pk = getattr(first, "_pack_owner", None)
        if pk is not None and pk.dtype == dtype and self.arena is not None:
            # the model-level pack: one pack_lora_multi launch per step for every group (no torch ops)
            self.A32s, self.B32, self.B32t, self.At32 = pk.multi(
                id(cat), cat.in_features, cat.out_features, [(l, n0, n1, q) for l, n0, n1, q in self.slots])
            return
        key = (self.arena.version if self.arena is not None else None, dtype, _PACK_GEN[0])
        cached = getattr(cat, "_mpack", None)
        if self.arena is not None and cached is not None and cached[0] == key:
            self.A32s, self.B32, self.B32t, self.At32 = cached[1]
            return
        K, N = cat.in_features, cat.out_features
        dev = first.lora_A.weight.device
        A_ext = torch.zeros(32, K, dtype=torch.float32, device=dev)
        B_ext = torch.zeros(N, 32, dtype=torch.float32, device=dev)
        Bt_ext = torch.zeros(32, N, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for l, n0, n1, q in self.slots:
                A, B, r, s = l.lora_A.weight.detach(), l.lora_B.weight.detach(), l.lora_r, l.lora_scaling
                A_ext[q:q + r] = A * s
                B_ext[n0:n1, q:q + r] = B
                Bt_ext[q:q + r, n0:n1] = B.t() * s
            At = torch.zeros(K, 32, dtype=torch.float32, device=dev)
            for l, n0, n1, q in self.slots:
                At[:, q:q + l.lora_r] = l.lora_A.weight.detach().t()
        self.A32s, self.B32 = A_ext.to(dtype), B_ext.to(dtype)
        self.B32t, self.At32 = Bt_ext.to(dtype), At.to(dtype)
        if self.arena is not None:
            cat._mpack = (key, (self.A32s, self.B32, self.B32t, self.At32))

    def forward(self, x, seed, training):
        return K.lora_proj(x, self.A32s, 1.0, self.p if training else 0.0, seed, rows=self.rows)

    def backward(self, gz, x, T32, seed, training, dT32=None):
        p = self.p if training else 0.0
        if dT32 is None:
            dT32 = K.lora_proj(gz, self.B32t, 1.0, 0.0, 0, rows=self.rows)
        grads = []
        if self.arena is not None:  # per-slot dB on gz's column span; ONE dA problem feeds every slot
            for l, n0, n1, q in self.slots:
                _WG.add(self.arena, gz[:, n0:n1], T32, 1, [(q, l.lora_r, l._offB)], 0.0, 0, (l._offB,))
            for i in range(0, len(self.slots), 4):
                grp = self.slots[i:i + 4]
                _WG.add(self.arena, x, dT32, 2, [(q, l.lora_r, l._offA) for l, _, _, q in grp], p, seed,
                        [l._offA for l, _, _, _ in grp])
            return [None, None] * len(self.slots), dT32
        dAf = K.lora_wgrad(x, dT32, p=p, seed=seed)
        for l, n0, n1, q in self.slots:
            dBf = K.lora_wgrad(gz[:, n0:n1], T32)
            grads += [dAf[:, q:q + l.lora_r].t(), dBf[:, q:q + l.lora_r]]
        return grads, dT32


def _flat(x):
    return x.reshape(-1, x.shape[-1])


def _dgrad(gz, lin, lo, dT32, seed, training, **kw):
    """dX = gz·W (+ LoRA K-extension under the LoRA-input dropout mask)."""
    if lo is None:
        return K.gemm(gz, lin.w_kn(), **kw)
    p = lo.p if training else 0.0
    return K.gemm(gz, lin.w_kn(), a2=dT32, b2=lo.At32, ext_p=p, ext_seed=seed, **kw)


def _nones(n):
    return [None] * n


# ---------------------------------------------------------------------------
class ResidualLink:
    """Carries the residual-stream gradient from ``linear_residual``'s backward to the
    ``ln_linear`` that read the same hidden state: h feeds both (LN -> qkv, and the residual
    add), and instead of autograd summing the two gradients with a separate add kernel, the
    residual part enters ``layer_norm_bwd`` as its ``dres`` operand (reverse order is
    guaranteed: the residual Function consumes the attention output, which depends on the LN
    branch)."""
    __slots__ = ("g",)

    def __init__(self):
        self.g = None


class GradHandoff:
    """An LN backward hands its output straight to the residual-dropout backward of the LoRA linear
    that produced the LN's input, in one row pass (K.ln_bwd_mask_proj, rowproj.hip MODE 3).

    The consumer (``linear_residual`` / ``mlp``: h' = h + dropout(lin(..)), LoRA on lin) registers its
    dropout (p, seed) and adapter in forward; the producer (the LN backward of the NEXT op in forward
    order, whose LN reads h') computes dh, y = dropout-bwd(dh) and dT0 = s·y·Bᵀ together and leaves
    (dh, y, dT0) here; the consumer's backward takes them when the gradient it receives IS that dh
    (same storage), else it runs its own mask_proj.  MIFT_LN_MASK_PROJ=0 turns the fusion off."""
    __slots__ = ("p", "seed", "lo", "out")

    def __init__(self):
        self.p, self.seed, self.lo, self.out = None, 0, None, None

    def register(self, p, seed, lo):
        self.p, self.seed, self.lo, self.out = p, seed, lo, None

    def ready(self, D):
        return (self.lo is not None and os.environ.get("MIFT_LN_MASK_PROJ", "1") != "0"
                and _mfma_width(D, "ln_bwd") and K.ln_bwd_mask_proj_ok(D))

    def ln_bwd(self, da, x2, ln_w, mean, rstd, dres):
        """LN backward (+ dres); with a registered consumer also its mask_proj, kept for it."""
        if not self.ready(x2.shape[-1]):
            return K.layer_norm_bwd(da, x2, ln_w, mean, rstd, dres=dres)[0]
        lo = self.lo
        dh, y, dT0 = K.ln_bwd_mask_proj(da, x2, ln_w, mean, rstd, dres, self.p, self.seed, lo.B32t, lo.rows,
                                        lo.dt_alpha)
        self.out = (dh, y, dT0)
        return dh

    def take(self, g2):
        """(y, dT0) computed for gradient g2 by the LN backward, or None."""
        out, self.out = self.out, None
        if out is None or out[0].data_ptr() != g2.data_ptr() or out[0].shape != g2.shape:
            return None
        return out[1], out[2]


def _ln_bwd(hand, da, x2, ln_w, mean, rstd, dres):
    if hand is not None:
        return hand.ln_bwd(da, x2, ln_w, mean, rstd, dres)
    return K.layer_norm_bwd(da, x2, ln_w, mean, rstd, dres=dres)[0]


def _mask_proj_in(hand, g2, p, seed, lo):
    """The consumer side of GradHandoff: the LN backward's (gz, dT0) for g2, or a mask_proj pass."""
    got = hand.take(g2) if hand is not None else None
    return got if got is not None else _mask_proj(g2, p, seed, lo)


class LnLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ln_w, ln_b, lin, eps, lora_seed, training, link, *lparams):
        shp = x.shape
        x2 = _flat(x.contiguous())
        lo = lin.lora_ops(x.dtype) if lparams else None
        if lo is not None:  # LN and the LoRA input projection in one row pass (csrc/kernels/rowproj.hip)
            a, mean, rstd, T32 = _ln_fwd_lora(x2, ln_w, ln_b, eps, lo, lora_seed, training)
        else:
            a, mean, rstd = K.layer_norm_fwd(x2, ln_w, ln_b, eps)
            T32 = None
        y = K.gemm(a, lin.w_nk(), lin.bias, T32, lo.B32 if lo else None)
        ctx.save_for_backward(x2, a, mean, rstd, ln_w, T32)
        ctx.lin, ctx.lo, ctx.seed, ctx.training, ctx.shp, ctx.nl = lin, lo, lora_seed, training, shp, len(lparams)
        ctx.link = link
        ctx.hand = getattr(x, "_mift_hand", None)  # the upstream mlp's dropout-bwd rides on this LN backward
        return y.view(*shp[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, gy):
        x2, a, mean, rstd, ln_w, T32 = ctx.saved_tensors
        lin, lo = ctx.lin, ctx.lo
        gy = _flat(gy.contiguous())
        lg, dT32 = (lo.backward(gy, a, T32, ctx.seed, ctx.training) if lo is not None else (_nones(ctx.nl), None))
        _WG.flush()  # the layer's first op in forward order: its adapters' weight grads, one launch
        gres = ctx.link.g if ctx.link is not None else None
        if ctx.link is not None:
            ctx.link.g = None
        if not ctx.needs_input_grad[0]:
            # e.g. the first block, fed by the frozen embedding: no dX -> no dgrad GEMM, no LN backward
            return (None, None, None, None, None, None, None, None, *lg)
        da = _dgrad(gy, lin, lo, dT32, ctx.seed, ctx.training)
        dx = _ln_bwd(ctx.hand, da, x2, ln_w, mean, rstd, None if gres is None else _flat(gres.contiguous()))
        return (dx.view(ctx.shp), None, None, None, None, None, None, None, *lg)


def _infer_ln_gemm(x, ln, lin):
    """No autograd, no adapter, <= 64 rows (greedy decode): LN inside the skinny GEMM, or None."""
    if torch.is_grad_enabled() or lin.lora_params() or x.numel() // x.shape[-1] > 64:
        return None
    x2 = _flat(x.contiguous())
    w = lin.w_nk()
    if not K.gemm_ln_ok(x2, w, ln.weight):
        return None
    return x2, w


def _ln_fold(ln, lin, w):
    """(wf, c1, c2) of LayerNorm(x; γ, β)·wᵀ + bias with the LN folded into the weights: wf = γ∘w rounded
    to w's dtype, c1 = Σ_k wf[:, k] and c2 = w·β + bias in fp32 (K.gemm_ln_fold).  Cached on the linear,
    keyed by the storage and version counters of the SOURCE parameters (each member linear's weight and
    bias, the LN's): ``w`` itself may be a derived cached tensor (a transpose / concatenation) whose
    rebuilt copy can land at the same address with version 0, so keying on it could reuse stale folds
    (ADVICE r5)."""
    b = lin.bias
    members = getattr(lin, "lins", None) or [lin]
    src = tuple((m.weight.data_ptr(), m.weight._version) if getattr(m, "weight", None) is not None else None
                for m in members)
    key = (src, w.data_ptr(), w._version, w.shape, ln.weight.data_ptr(), ln.weight._version, ln.bias.data_ptr(),
           ln.bias._version, None if b is None else (b.data_ptr(), b._version))
    c = getattr(lin, "_mift_lnfold", None)
    if c is None or c[0] != key:
        g, beta = ln.weight.detach().float(), ln.bias.detach().float()
        wf = (w.float() * g[None, :]).to(w.dtype).contiguous()
        c1 = wf.float().sum(1).contiguous()
        c2 = (w.float() @ beta + (b.detach().float() if b is not None else 0.0)).contiguous()
        c = (key, wf, c1, c2)
        lin._mift_lnfold = c
    return c[1:]


def _gemm_ln(x2, ln, lin, w, act=0):
    """Decode projection of LN(x): the folded form (K.gemm_ln_fold) unless MIFT_LN_FOLD=0 (read per call:
    the LN-prologue form, K.gemm_ln).  Both are M <= 64 skinny-GEMM launches."""
    if os.environ.get("MIFT_LN_FOLD", "1") != "0":
        wf, c1, c2 = _ln_fold(ln, lin, w)
        return K.gemm_ln_fold(x2, wf, c1, c2, ln.eps, act=act)
    return K.gemm_ln(x2, ln.weight, ln.bias, ln.eps, w, lin.bias, act=act)


def ln_linear(x, ln, lin, lora_seed=0, training=True, link=None):
    fast = _infer_ln_gemm(x, ln, lin)
    if fast is not None:  # decode: one launch instead of LN + GEMM
        x2, w = fast
        return _gemm_ln(x2, ln, lin, w).view(*x.shape[:-1], w.shape[0])
    return LnLinear.apply(x, ln.weight, ln.bias, lin, ln.eps, lora_seed, training, link, *lin.lora_params())


# ---------------------------------------------------------------------------
class LinearResidual(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h, lin, p, seed, lora_seed, training, link, hand, *lparams):
        shp = h.shape
        x2 = _flat(x.contiguous())
        h2 = _flat(h.contiguous())
        lo = lin.lora_ops(x.dtype) if lparams else None
        T32 = lo.forward(x2, lora_seed, training) if lo is not None else None
        pp = p if training else 0.0
        y = K.gemm(x2, lin.w_nk(), lin.bias, T32, lo.B32 if lo else None, residual=h2, dropout_p=pp, seed=seed)
        ctx.save_for_backward(x2, T32)
        ctx.lin, ctx.lo, ctx.p, ctx.seed, ctx.lseed = lin, lo, pp, seed, lora_seed
        ctx.training, ctx.xshp, ctx.nl, ctx.link = training, x.shape, len(lparams), link
        ctx.hand = hand
        if hand is not None:
            hand.register(pp, seed, lo)
        return y.view(shp)

    @staticmethod
    def backward(ctx, gh):
        x2, T32 = ctx.saved_tensors
        lin, lo = ctx.lin, ctx.lo
        gh2 = _flat(gh.contiguous())
        if lo is not None:  # residual-dropout backward and dT = s·gz·B in one row pass
            gz, dT0 = _mask_proj_in(ctx.hand, gh2, ctx.p, ctx.seed, lo)
            lg, dT32 = lo.backward(gz, x2, T32, ctx.lseed, ctx.training, dT32=dT0)
        else:
            gz = K.mask_scale(gh2, ctx.p, ctx.seed) if ctx.p > 0 else gh2
            lg, dT32 = _nones(ctx.nl), None
        dx = _dgrad(gz, lin, lo, dT32, ctx.lseed, ctx.training)
        gres = gh
        if ctx.link is not None and ctx.needs_input_grad[1]:
            ctx.link.g, gres = gh, None  # delivered through the linked ln_linear's LN backward
        return (dx.view(ctx.xshp), gres, None, None, None, None, None, None, None, *lg)


def linear_residual(x, h, lin, p, seed, lora_seed=0, training=True, link=None, handoff=None):
    """h + dropout(lin(x)); ``handoff`` (GradHandoff): the following LN backward also runs this
    op's residual-dropout backward + dT projection."""
    return LinearResidual.apply(x, h, lin, p, seed, lora_seed, training, link, handoff, *lin.lora_params())


# ---------------------------------------------------------------------------
class MLP(torch.autograd.Function):
    """h' = h + dropout(fc2(act(fc1(LN(h)))))."""

    @staticmethod
    def forward(ctx, h, ln_w, ln_b, fc1, fc2, eps, act, p, seed, seed_l1, seed_l2, training, n1, hand_out, hand_in,
                *lparams):
        shp = h.shape
        h2 = _flat(h.contiguous())
        lo1 = fc1.lora_ops(h.dtype) if n1 else None
        lo2 = fc2.lora_ops(h.dtype) if len(lparams) > n1 else None
        if lo1 is not None:  # LN and fc1's LoRA input projection in one row pass (OPT targets fc1)
            a, mean, rstd, T1 = _ln_fwd_lora(h2, ln_w, ln_b, eps, lo1, seed_l1, training)
        else:
            a, mean, rstd = K.layer_norm_fwd(h2, ln_w, ln_b, eps)
            T1 = None
        # fc2's LoRA input projection T2 = s·drop(f)·A2ᵀ comes out of the fc1 epilogue (per column
        # tile partials + one ordered reduction) instead of a lora_proj pass re-reading f
        pk = _epi_proj_kw(lo2, seed_l2, training)
        if act == 2:  # ReLU: relu'(z) = [f > 0], so f doubles as the backward's aux (no pre-activation store)
            # ... or, 16x fewer bytes for the dgrad epilogue to read, the sign bits of f (MIFT_RELU_BITS=0: f)
            N1 = fc1.w_nk().shape[0]
            bits = (torch.empty(h2.shape[0], N1 // 8, dtype=torch.uint8, device=h2.device)
                    if N1 % 8 == 0 and os.environ.get("MIFT_RELU_BITS", "1") != "0" else None)
            r = K.gemm(a, fc1.w_nk(), fc1.bias, T1, lo1.B32 if lo1 else None, act=act, sbits=bits, **pk)
            f, T2 = r if pk else (r, None)
            z = f if bits is None else bits
        else:
            r = K.gemm(a, fc1.w_nk(), fc1.bias, T1, lo1.B32 if lo1 else None, act=act, want_preact=True, **pk)
            f, z, T2 = r if pk else r + (None,)
        if lo2 is not None and T2 is None:
            T2 = lo2.forward(f, seed_l2, training)
        pp = p if training else 0.0
        out = K.gemm(f, fc2.w_nk(), fc2.bias, T2, lo2.B32 if lo2 else None, residual=h2, dropout_p=pp, seed=seed)
        ctx.save_for_backward(h2, a, mean, rstd, ln_w, z, f, T1, T2)
        ctx.fc1, ctx.fc2, ctx.lo1, ctx.lo2 = fc1, fc2, lo1, lo2
        ctx.act, ctx.p, ctx.seed, ctx.sl1, ctx.sl2, ctx.training, ctx.shp = act, pp, seed, seed_l1, seed_l2, training, shp
        ctx.n1, ctx.n2 = n1, len(lparams) - n1
        ctx.hand_out, ctx.hand_in = hand_out, hand_in
        if hand_in is not None:
            hand_in.register(pp, seed, lo2)
        return out.view(shp)

    @staticmethod
    def backward(ctx, gh):
        h2, a, mean, rstd, ln_w, z, f, T1, T2 = ctx.saved_tensors
        fc1, fc2, lo1, lo2 = ctx.fc1, ctx.fc2, ctx.lo1, ctx.lo2
        gh2 = _flat(gh.contiguous())
        lg1, lg2 = _nones(ctx.n1), _nones(ctx.n2)
        dT1 = dT2 = None
        if lo2 is not None:  # residual-dropout backward fused with dT2 = s·gm·B2
            gm, dT0 = _mask_proj_in(ctx.hand_in, gh2, ctx.p, ctx.seed, lo2)
            lg2, dT2 = lo2.backward(gm, f, T2, ctx.sl2, ctx.training, dT32=dT0)
        else:
            gm = K.mask_scale(gh2, ctx.p, ctx.seed) if ctx.p > 0 else gh2
        # dZ = (gm·W2 [+ masked LoRA ext]) ⊙ act'(z), all in the dgrad epilogue — which also emits fc1's
        # adapter projection dT1 = s·dZ·B1 from the dZ tile it just wrote (OPT targets fc1)
        pk = _epi_dt_kw(lo1)
        if z.dtype == torch.uint8:  # ReLU sign bits of f (forward)
            r = _dgrad(gm, fc2, lo2, dT2, ctx.sl2, ctx.training, act=_BWD[ctx.act], sbits=z, **pk)
        else:
            r = _dgrad(gm, fc2, lo2, dT2, ctx.sl2, ctx.training, act=_BWD[ctx.act], aux=z, **pk)
        dz, dT1e = r if pk else (r, None)
        if lo1 is not None:
            lg1, dT1 = lo1.backward(dz, a, T1, ctx.sl1, ctx.training, dT32=dT1e)
        da = _dgrad(dz, fc1, lo1, dT1, ctx.sl1, ctx.training)
        dh = _ln_bwd(ctx.hand_out, da, h2, ln_w, mean, rstd, gh2)
        return (dh.view(ctx.shp),) + (None,) * 14 + tuple(lg1) + tuple(lg2)


def mlp(h, ln, fc1, fc2, act, p, seed, seed_l1=0, seed_l2=0, training=True, handoff=None):
    """h + dropout(fc2(act(fc1(LN(h))))).  ``handoff``: this op's LN backward also runs the residual-dropout
    backward of the linear_residual that produced h; the output carries a GradHandoff of its own for the
    next block's ln_linear (attribute ``_mift_hand``)."""
    fast = _infer_ln_gemm(h, ln, fc1)
    if fast is not None and not training:  # decode: LN inside fc1's skinny GEMM, no pre-activation store
        h2, w1 = fast
        f = _gemm_ln(h2, ln, fc1, w1, act=act)
        lo2 = fc2.lora_ops(h.dtype) if fc2.lora_params() else None
        T2 = lo2.forward(f, seed_l2, False) if lo2 is not None else None
        out = K.gemm(f, fc2.w_nk(), fc2.bias, T2, lo2.B32 if lo2 else None, residual=h2)
        return out.view(h.shape)
    l1, l2 = fc1.lora_params(), fc2.lora_params()
    hand_in = GradHandoff() if (training and l2 and torch.is_grad_enabled()) else None
    out = MLP.apply(h, ln.weight, ln.bias, fc1, fc2, ln.eps, act, p, seed, seed_l1, seed_l2, training, len(l1),
                    handoff, hand_in, *l1, *l2)
    if hand_in is not None:
        out._mift_hand = hand_in
    return out


# ---------------------------------------------------------------------------
class LMHeadXent(torch.autograd.Function):
    """Sum of token CE of LN(h) @ E^T against (already shifted) labels — the fused head.

    Forward (``lmhead_fwd``, csrc/kernels/gemm.hip EPI 1): the phased 256x256 MFMA GEMM keeps the
    logits in registers and writes E = exp(z - m_tile) per 256-column tile plus the tile
    statistics; the loss comes from those statistics (``lmhead_lse_kernel``).  Backward
    (``lmhead_dgrad``, EPI 2): dX = g·(softmax - onehot)·W as a split-K GEMM over E whose
    per-row, per-tile factors g·exp(m_tile - lse) are applied to group accumulators, the
    one-hot part subtracted in the split-K reduction — dlogits are never materialised, the
    upstream gradient is applied in fp32.  Reference loss head:
    ``Cluster/Project 2 - Course Project/finetune_lora_opt_pp.py:138-153``.

    ``MIFT_LMHEAD=blas`` selects the previous library path (hipBLASLt logits + xent kernel +
    hipBLASLt dgrad) for A/B measurements.

    No torch kernels around the two launches: the ignored id (OPT's pad) is masked inside the
    kernels, the loss sum comes out of ``lmhead_lse_kernel`` (deterministic in-launch reduction,
    ``_lm_ws``), and a replayed step's 1/tokens factor (``head_grad_mul``) is multiplied into the
    upstream gradient inside the dgrad reduction — VERDICT r3 hygiene (the per-step fill / binary /
    reduce / copy kernels of the graph)."""

    @staticmethod
    def forward(ctx, h, ln_w, ln_b, eps, w_nk, labels, V, ignore_index, need_grad, w_kn, shift):
        shp = h.shape
        h2 = _flat(h.contiguous())
        a, mean, rstd = K.layer_norm_fwd(h2, ln_w, ln_b, eps)
        lab = labels.reshape(-1).contiguous()
        ign = int(ignore_index) if ignore_index >= 0 else -1  # e.g. OPT ignores the pad id, a real entry
        ctx.shp, ctx.w_nk, ctx.w_kn, ctx.V, ctx.shift, ctx.ign = shp, w_nk, w_kn, V, shift, ign
        ctx.hand = getattr(h, "_mift_hand", None)  # the last block's mlp dropout-bwd rides on the final LN's
        ctx.gmul = _HEAD_GMUL[0]
        if ctx.gmul is not None:
            _HEAD_GMUL[1] = True
        C = _lm_chunk(a.shape[0], shift) if need_grad else 0
        if C:
            # chunked: per C-row chunk the forward's E [C, V_pad] is consumed by that chunk's
            # dgrad at once (g = 1; the upstream gradient scales dX in backward), so no [T, V] tensor
            # lives past its chunk and the chunk's E can stay in the Infinity Cache
            w_kn_ = w_kn if w_kn is not None else w_nk.t().contiguous()
            one = _lm_one(a.device)
            ws = _lm_ws(a.device)
            dx, total = [], None
            for r0 in range(0, a.shape[0], C):
                ac, lc = a[r0:r0 + C], lab[r0:r0 + C]
                outs = K.lmhead_fwd(ac, w_nk, lc, V, shift, ign, ws)
                dx.append(K.lmhead_dgrad(outs[0], w_kn_, w_nk, lc, V, outs[1], outs[2], one, shift, ign, None))
                total = outs[5] if total is None else total + outs[5]
            ctx.save_for_backward(h2, mean, rstd, ln_w, torch.cat(dx))
            ctx.chunked = True
            return total.view(())
        outs = K.lmhead_fwd(a, w_nk, lab, V, shift, ign, _lm_ws(a.device))
        E, stats, lse, total = outs[0], outs[1], outs[2], outs[5]
        if need_grad:
            ctx.save_for_backward(h2, mean, rstd, ln_w, E, stats, lse, lab)
        ctx.chunked = False
        return total.view(())

    @staticmethod
    def backward(ctx, g):
        if ctx.chunked:
            h2, mean, rstd, ln_w, dx1 = ctx.saved_tensors
            sc = g.reshape(1).float() if ctx.gmul is None else g.reshape(1).float() * ctx.gmul
            da = (dx1.float() * sc).to(dx1.dtype)  # unit-gradient dX, scaled once in fp32
        else:
            h2, mean, rstd, ln_w, E, stats, lse, lab = ctx.saved_tensors
            w_kn = ctx.w_kn if ctx.w_kn is not None else ctx.w_nk.t().contiguous()
            g1 = g.reshape(1)
            da = K.lmhead_dgrad(E, w_kn, ctx.w_nk, lab, ctx.V, stats, lse,
                                g1 if g1.dtype == torch.float32 else g1.float(), ctx.shift, ctx.ign, ctx.gmul)
        dh = _ln_bwd(ctx.hand, da, h2, ln_w, mean, rstd, None)
        return dh.view(ctx.shp), None, None, None, None, None, None, None, None, None, None


class LMHeadXentBlas(torch.autograd.Function):
    """Library path (hipBLASLt logits, xent kernel rewrites them as dlogits, hipBLASLt dgrad)."""

    @staticmethod
    def forward(ctx, h, ln_w, ln_b, eps, w_nk, labels, V, ignore_index, need_grad):
        shp = h.shape
        h2 = _flat(h.contiguous())
        a, mean, rstd = K.layer_norm_fwd(h2, ln_w, ln_b, eps)
        M = a.shape[0]
        lab = labels.reshape(-1)
        chunk = _xent_chunk(M, w_nk.shape[0])
        if chunk >= M:
            logits = torch.matmul(a, w_nk.t())
            loss_rows, _ = K.xent(logits, lab, V, ignore_index, write_grad=need_grad)
        else:
            logits = torch.empty(M, w_nk.shape[0], dtype=a.dtype, device=a.device)
            loss_rows = torch.empty(M, dtype=torch.float32, device=a.device)
            for r0 in range(0, M, chunk):
                r1 = min(M, r0 + chunk)
                lg = logits[r0:r1]
                torch.matmul(a[r0:r1], w_nk.t(), out=lg)
                loss_rows[r0:r1] = K.xent(lg, lab[r0:r1], V, ignore_index, write_grad=need_grad)[0]
        if need_grad:
            ctx.save_for_backward(h2, mean, rstd, ln_w, logits)
        ctx.shp, ctx.w_nk = shp, w_nk
        return loss_rows.sum()

    @staticmethod
    def backward(ctx, g):
        h2, mean, rstd, ln_w, dlogits = ctx.saved_tensors
        da = torch.matmul(dlogits, ctx.w_nk)
        da = (da.float() * g.reshape(1).float()).to(dlogits.dtype)  # upstream grad applied in fp32
        dh, _, _, _ = K.layer_norm_bwd(da, h2, ln_w, mean, rstd)
        return dh.view(ctx.shp), None, None, None, None, None, None, None, None


_LM_WS = {}
_LM_ONE = {}


def _lm_chunk(M, shift):
    """Rows per chunk of the chunked head (MIFT_LM_CHUNK, read per call; 0 = whole batch, the default): a
    multiple of the sequence length when the labels are unshifted ids, and only when it actually splits M.
    Opt-in for memory-limited runs: the whole-batch head streams its 824 MB E once through HBM, which on
    MI355X costs less than the chunks' smaller grids and split-K slabs — distilgpt2 step 4.90 ms whole vs
    5.03 / 5.42 / 6.00 at 4096- / 2048- / 1024-row chunks (profiles/r5/step_ab_lm_chunk.json)."""
    c = int(os.environ.get("MIFT_LM_CHUNK", "0"))
    if c <= 0 or c >= M:
        return 0
    if shift:
        c = max(shift, c // shift * shift)
    return c if c < M else 0


def _lm_one(dev):
    """A device fp32 1.0 (the chunked head's dgrad runs at unit upstream gradient)."""
    t = _LM_ONE.get(dev)
    if t is None:
        t = _LM_ONE[dev] = torch.ones(1, dtype=torch.float32, device=dev)
    return t
_HEAD_GMUL = [None, False]  # (multiplier tensor, consumed by a head since set_head_grad_mul)


def _lm_ws(dev):
    """Per-device zero-initialised arrival counter of the LM head's in-launch loss reduction
    (self-resetting; the head's launches on a device are stream-ordered).  Created by the first
    (eager, warm-up) call, never inside a graph capture."""
    ws = _LM_WS.get(dev)
    if ws is None:
        ws = _LM_WS[dev] = torch.zeros(K.ARRIVE_INTS, dtype=torch.int32, device=dev)
    return ws


def set_head_grad_mul(t):
    """Make the next fused LM heads multiply their upstream gradient by the fp32 device scalar ``t``
    (None: off).  The graph-captured step passes its per-step 1/tokens here and seeds backward with
    the bare loss scale; ``head_grad_mul_used()`` tells whether a head took it (else the caller
    must scale the seed itself)."""
    _HEAD_GMUL[0], _HEAD_GMUL[1] = t, False


def head_grad_mul_used():
    return _HEAD_GMUL[1]


def _xent_chunk(M, Vp):
    """Rows per LM-head chunk (``MIFT_XENT_CHUNK``, default 0 = unchunked).

    Measured on MI355X (distilgpt2, M = 8192, V_pad = 50304): chunks of 768 / 1024 / 2048 / 4096
    rows ran 6.38 / 6.28 / 6.21 / 6.10 ms per step vs 5.99 unchunked — the smaller hipBLASLt GEMMs
    lose more than the cache-resident xent pass gains, so chunking is opt-in (large-vocab,
    memory-limited runs)."""
    import os
    c = int(os.environ.get("MIFT_XENT_CHUNK", "0"))
    return M if c <= 0 or c >= M else c


def lm_head_xent(h, ln, w_nk, labels, V, ignore_index=-100, need_grad=True, w_kn=None, shift=0):
    """Summed token CE.  ``labels``: per-row targets (shift = 0) or, with ``shift = S``, the unshifted
    [B, S] ids (row r's target is ids[r + 1] within its sequence, none at a sequence's end)."""
    if os.environ.get("MIFT_LMHEAD", "fused") == "blas":
        if shift:
            from ..models.base import shift_labels
            labels = shift_labels(labels.reshape(-1, shift), ignore_index)
        return LMHeadXentBlas.apply(h, ln.weight, ln.bias, ln.eps, w_nk, labels, V, ignore_index, need_grad)
    return LMHeadXent.apply(h, ln.weight, ln.bias, ln.eps, w_nk, labels, V, ignore_index, need_grad, w_kn,
                            int(shift))


def lm_head_logits(h, ln, w_nk, V):
    """Logits of the tied head (inference / generation): LN kernel + the MFMA ``gemm_nt`` against
    the padded [V_pad, d] weight — no library GEMM on the decode path."""
    h2 = _flat(h.contiguous())
    a, _, _ = K.layer_norm_fwd(h2, ln.weight, ln.bias, ln.eps)
    logits = K.gemm(a, w_nk)
    return logits[:, :V].reshape(*h.shape[:-1], V)
