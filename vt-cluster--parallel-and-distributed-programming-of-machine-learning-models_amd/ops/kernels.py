"""Thin, keyword-friendly wrappers over ``mift._C`` (GPU tensors only).

Every wrapper launches on torch's current HIP stream.  CPU callers use
``mift.ops.reference`` instead (see ``mift.ops.dispatch``).
"""
from .dispatch import C

ACT = {"none": 0, "gelu_new": 1, "gelu_tanh": 1, "relu": 2, "gelu": 3, "gelu_erf": 3}
ACT_BWD = {0: 0, 1: 4, 2: 5, 3: 6}


def gemm(a, b, bias=None, a2=None, b2=None, act=0, aux=None, residual=None, dropout_p=0.0, seed=0,
         want_preact=False, alpha=1.0, out=None, tile=0, alpha_t=None, pre_add=None):
    """out = epi(a @ b.T [+ a2 @ b2.T]); see csrc/kernels/gemm.hip."""
    y, pre = C().gemm_nt(a, b, bias, a2, b2, int(act), aux, residual, float(dropout_p), int(seed),
                         bool(want_preact), float(alpha), out, int(tile), alpha_t, pre_add)
    return (y, pre) if want_preact else y


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


def pack_lora(A, B, a_scale, dtype):
    return C().pack_lora(A, B, float(a_scale), dtype)


def xent(logits, labels, V, ignore_index=-100, write_grad=True):
    return C().xent_fwd_bwd(logits, labels, int(V), int(ignore_index), bool(write_grad))
