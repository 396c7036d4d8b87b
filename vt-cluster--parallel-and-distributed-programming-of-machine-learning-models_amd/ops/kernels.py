"""Thin, keyword-friendly wrappers over ``mift._C`` (GPU tensors only).

Every wrapper launches on torch's current HIP stream.  CPU callers use
``mift.ops.reference`` instead (see ``mift.ops.dispatch``).
"""
import torch

from .dispatch import C

ACT = {"none": 0, "gelu_new": 1, "gelu_tanh": 1, "relu": 2, "gelu": 3, "gelu_erf": 3}
ACT_BWD = {0: 0, 1: 4, 2: 5, 3: 6}


def gemm(a, b, bias=None, a2=None, b2=None, act=0, aux=None, residual=None, dropout_p=0.0, seed=0,
         want_preact=False, alpha=1.0, out=None, tile=0, alpha_t=None, pre_add=None, ext_p=0.0, ext_seed=0,
         proj_w=None, proj_rows=32, proj_p=0.0, proj_seed=0, proj_alpha=1.0, sbits=None):
    """out = epi(a @ b.T [+ a2 @ b2.T]); see csrc/kernels/gemm.hip.

    ``ext_p > 0`` keeps the a2·b2ᵀ K-extension separate and adds it under the
    dropout mask (ext_seed, ext_p) — the LoRA input-dropout backward.
    ``proj_w`` ([32, N], first ``proj_rows`` rows non-zero): also return
    T = proj_alpha · dropout(out; proj_p, proj_seed) @ proj_w.T [M, 32] computed in the epilogue
    (= lora_proj(out, proj_w, proj_alpha, proj_p, proj_seed) without re-reading out).
    ``sbits`` (uint8 [M, N/8]): with ``act`` = ReLU the epilogue writes the sign bits of the stored
    output into it; with the ReLU backward (``act`` = 5, no ``aux``) it reads them as the mask."""
    y, pre, t = C().gemm_nt(a, b, bias, a2, b2, int(act), aux, residual, float(dropout_p), int(seed),
                            bool(want_preact), float(alpha), out, int(tile), alpha_t, pre_add, float(ext_p),
                            int(ext_seed), proj_w, int(proj_rows), float(proj_p), int(proj_seed), float(proj_alpha),
                            sbits)
    res = (y, pre) if want_preact else (y,)
    if proj_w is not None:
        res = res + (t,)
    return res if len(res) > 1 else y


def gemm_ln_ok(x, w, ln_w):
    """The LN-prologue skinny GEMM applies: <= 64 rows (decode), narrow N, K <= 1024, one dtype."""
    M, K = x.shape
    return (x.is_cuda and x.dtype == w.dtype == ln_w.dtype and x.stride(1) == 1
            and C().gemm_ln_ok(int(M), int(w.shape[0]), int(K)))


def gemm_ln(x, ln_w, ln_b, eps, w, bias=None, act=0, want_preact=False):
    """act(LayerNorm(x) @ w.T + bias) in one launch (M <= 64: the decode projections)."""
    y, pre = C().gemm_ln(x, ln_w, ln_b, float(eps), w, bias, int(act), bool(want_preact))
    return (y, pre) if want_preact else y


def gemm_ln_fold(x, wf, c1, c2, eps, act=0):
    """act(LayerNorm(x) @ w.T + bias) with the LN folded into the weights (wf = γ∘w, c1 = wf row sums,
    c2 = w·β + bias, fp32): rstd·(x @ wf.T − mean·c1) + c2 in one launch (M <= 64, decode)."""
    return C().gemm_ln_fold(x, wf, c1, c2, float(eps), int(act))


def lora_proj(x, w32, alpha=1.0, p=0.0, seed=0, rows=32):
    """[M,32] = alpha * dropout(x) @ w32.T   (w32: [32, K]; only its first ``rows`` rows may be non-zero)."""
    return C().lora_proj(x, w32, float(alpha), float(p), int(seed), int(rows))


def lora_wgrad(x, y32, out=None, p=0.0, seed=0):
    """out[P,32] (fp32) += dropout(x).T @ y32."""
    import torch
    if out is None:
        out = torch.zeros(x.shape[1], 32, dtype=torch.float32, device=x.device)
    C().lora_wgrad(x, y32, out, float(p), int(seed), 0, 32, 0, 0)
    return out


def lora_wgrad_group(out, xs, ys, meta, ps):
    """Grouped weight grads (one launch, <= 16 problems) into the flat fp32 ``out``;
    meta: per problem [mode, nslot, (qoff, rank, offset) x 4, seed] (csrc/kernels/lora.hip)."""
    C().lora_wgrad_group(out, list(xs), list(ys), [int(v) for v in meta], [float(v) for v in ps])


def lora_wgrad_into(x, y32, arena_grad, mode, rank, offset, p=0.0, seed=0, qoff=0):
    """Accumulate dropout(x).T @ y32 into a flat fp32 arena: mode 1 -> [P, rank] (dB), 2 -> [rank, P] (dA)."""
    C().lora_wgrad(x, y32, arena_grad, float(p), int(seed), int(mode), int(rank), int(offset), int(qoff))


def layer_norm_fwd(x, w, b, eps):
    return C().layer_norm_fwd(x, w, b, float(eps))


def layer_norm_bwd(dy, x, w, mean, rstd, dres=None, branch_p=None, seed=0, want_wgrad=False):
    dx, dbr, dw, db = C().layer_norm_bwd(dy, x, w, mean, rstd, dres, branch_p is not None,
                                         float(branch_p or 0.0), int(seed), bool(want_wgrad))
    return dx, (dbr if branch_p is not None else None), (dw if want_wgrad else None), (db if want_wgrad else None)


def mask_scale(x, p, seed, out=None, accumulate=False):
    return C().mask_scale(x, float(p), int(seed), out, bool(accumulate))


def act_bwd(g, z, act, p=0.0, seed=0):
    return C().act_bwd(g, z, int(act), float(p), int(seed))


def embed(ids, wte, wpe=None, pos=None, pos_offset=0, p=0.0, seed=0):
    return C().embed_fwd(ids, pos, wte, wpe, int(pos_offset), float(p), int(seed), wte.dtype)


def mask_positions(mask):
    """(cumsum(mask)·mask - 1 [B, S] int64, Σ mask [B] int32) of an int64 [B, S] attention mask."""
    return C().mask_positions(mask)


def pack_lora(A, B, a_scale, dtype):
    return C().pack_lora(A, B, float(a_scale), dtype)


# int32 words of one in-launch arrival-counter set (csrc/common.h MIFT_ARRIVE_INTS: 8 group counters
# + 1 top counter, one 128-B line each); the kernels check the size they are given
ARRIVE_INTS = 9 * 32


def lmhead_fwd(a, w_nk, labels, V, shift=0, ignore_index=-1, ws=None):
    """Fused LM head + CE forward -> (E, stats, lse, loss_rows, zlab[, total]); labels outside [0, V)
    and ``ignore_index`` (>= 0) are no target.  ``shift = S``: labels are the unshifted ids of length-S
    sequences (row r's target is ids[r + 1]).  ``ws`` (int32[ARRIVE_INTS], zero, stream-ordered users): the
    kernel also returns the summed loss ``total`` [1] (deterministic in-launch reduction)."""
    return C().lmhead_fwd(a, w_nk, labels, int(V), int(shift), int(ignore_index), ws)


def lmhead_dgrad(E, w_kn, w_nk, labels, V, stats, lse, gscale, shift=0, ignore_index=-1, gmul=None):
    """dX = g·(softmax - onehot)·W from the forward's E / tile stats (no dlogits); g = gscale[0]
    (x gmul[0] when given)."""
    return C().lmhead_dgrad(E, w_kn, w_nk, labels, int(V), stats, lse, gscale, int(shift), int(ignore_index), gmul)


def xent(logits, labels, V, ignore_index=-100, write_grad=True):
    return C().xent_fwd_bwd(logits, labels, int(V), int(ignore_index), bool(write_grad))


def decode_tail(logits, V, done, ids, out, col, pos, t, fill, pad, eos):
    """One launch per greedy decode step (csrc/kernels/decode.hip): token = argmax(logits[b, :V])
    (first maximal index), ``pad`` for finished rows, out[b, col[b]] = token, done |= token == eos
    (eos None: never), ids[b] = done ? fill : token, col / pos / t += 1 — all in place."""
    C().decode_tail(logits, int(V), done, ids, out, col, pos, t, int(fill), int(pad),
                    -1 if eos is None else int(eos))


def kv_store(qkv, kcache, vcache, S):
    """Prefill: rows [0, S) of every (b, h) of the caches [B, H, Tmax, hd] from qkv [B*S, 3*H*hd]."""
    C().kv_store(qkv, kcache, vcache, int(S))


def decode_attn(qkv, kcache, vcache, t, scale, start=None, plen=None, gend=0):
    """o [B, H*hd] for the token at position t; writes its k/v into the caches.  Masked keys:
    ``< start[b]`` (left padding) and ``[plen[b], gend)`` (right-aligned prompts, generate.py).
    ``t`` may be an int32 [1] device tensor (graph-replayed decode: the position advances in-graph)."""
    if isinstance(t, torch.Tensor):
        return C().decode_attn(qkv, kcache, vcache, int(gend), float(scale), start, plen, int(gend), t)
    return C().decode_attn(qkv, kcache, vcache, int(t), float(scale), start, plen, int(gend), None)


def layer_norm_fwd_proj(x, w, b, eps, pw, rank, alpha=1.0, p=0.0, seed=0):
    """(y, mean, rstd, proj[M,32]) = LN(x), alpha·dropout(y)·pwᵀ — LN fused with the LoRA projection."""
    return C().layer_norm_fwd_proj(x, w, b, float(eps), pw, int(rank), float(alpha), float(p), int(seed))


def ln_bwd_mask_proj_ok(D):
    return bool(C().ln_bwd_mask_proj_ok(int(D)))


def ln_bwd_mask_proj(dy, x, w, mean, rstd, dres, p, seed, pw, rank, alpha=1.0):
    """(dh, y, proj): dh = layer_norm_bwd(dy; x, w, mean, rstd) + dres, then mask_proj(dh, p, seed, pw, rank,
    alpha) in the same row pass (csrc/kernels/rowproj.hip MODE 3)."""
    return C().ln_bwd_mask_proj(dy, x, w, mean, rstd, dres, float(p), int(seed), pw, int(rank), float(alpha))


def mask_proj(x, p, seed, pw, rank, alpha=1.0):
    """(y, proj[M,32]) = dropout(x) (x itself when p == 0), alpha·y·pwᵀ — dropout-bwd fused with dT."""
    return C().mask_proj(x, float(p), int(seed), pw, int(rank), float(alpha))
