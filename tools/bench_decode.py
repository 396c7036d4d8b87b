"""Per-op timings of the greedy decode step's kernels at distilgpt2 batch 64 (M = 64 rows), alone.

  python tools/bench_decode.py [--json out.json]

decode_tail (argmax + bookkeeping over 64 x 50257 logits), the LN-prologue skinny GEMMs (c_attn,
c_fc), the skinny c_proj, fc2 and the LM head on their default paths — to separate kernel time from
in-graph effects in the decode trace (profiles/r4/decode_skinny*_trace.txt)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import mift  # noqa: E402
from mift.ops import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    mift._ext.require()
    dt, dev, B, d, V, Vp = torch.bfloat16, "cuda", 64, 768, 50257, 50304
    torch.manual_seed(0)
    rows = []

    def rec(name, fn, **kw):
        t = timeit(fn)
        row = {"name": name, "us": round(t * 1e3, 2), **kw}
        print(json.dumps(row), flush=True)
        rows.append(row)

    logits = torch.randn(B, Vp, device=dev).to(dt)[:, :V]
    done = torch.zeros(B, dtype=torch.bool, device=dev)
    ids = torch.zeros(B, 1, dtype=torch.long, device=dev)
    out = torch.zeros(B, 16, dtype=torch.long, device=dev)
    col = torch.zeros(B, 1, dtype=torch.long, device=dev)
    pos = torch.zeros(B, 1, dtype=torch.long, device=dev)
    t = torch.zeros(1, dtype=torch.int32, device=dev)

    def tail():
        col.zero_()
        K.decode_tail(logits, V, done, ids, out, col, pos, t, 0, 50256, 50256)

    for nth in ("256", "512", "1024"):
        os.environ["MIFT_TAIL_NTH"] = nth
        rec(f"decode_tail(+col reset) {nth} threads", tail)
    os.environ.pop("MIFT_TAIL_NTH")
    rec("decode_tail(+col reset)", tail)
    # the tail's last steps alone: one row's argmax over 64 columns (bookkeeping-bound)
    rec("decode_tail V=64 (bookkeeping only)", lambda: (col.zero_(), K.decode_tail(logits, 64, done, ids, out, col, pos,
                                                                                   t, 0, 50256, 50256)))
    rec("col reset alone", lambda: col.zero_())
    rec("torch argmax (float)", lambda: logits.float().argmax(-1))
    x = torch.randn(B, d, device=dev).to(dt)
    lw = torch.ones(d, device=dev, dtype=dt)
    lb = torch.zeros(d, device=dev, dtype=dt)
    for name, N, Kd, act in (("c_attn", 3 * d, d, 0), ("c_fc", 4 * d, d, 1)):
        w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).to(dt)
        bias = torch.zeros(N, device=dev, dtype=dt)
        rec(f"gemm_ln {name} {B}x{N}x{Kd}", lambda: K.gemm_ln(x, lw, lb, 1e-5, w, bias, act=act))
        rec(f"ln + gemm {name}", lambda: K.gemm(K.layer_norm_fwd(x, lw, lb, 1e-5)[0], w, bias, act=act))
    for name, N, Kd in (("attn.c_proj", d, d), ("mlp.c_proj", d, 4 * d), ("lm_head", Vp, d)):
        xa = torch.randn(B, Kd, device=dev).to(dt)
        w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).to(dt)
        rec(f"gemm {name} {B}x{N}x{Kd}", lambda: K.gemm(xa, w))
        rec(f"gemm {name} tile4", lambda: K.gemm(xa, w, tile=4))
    # epilogue-operand prefetch A/B (MIFT_SKINNY_PF, read per call) on the decode epilogues: bias (+gelu)
    # for the LN-prologue GEMMs, bias + residual for c_proj / fc2 (K split 3)
    res = torch.randn(B, d, device=dev).to(dt)
    cases = []
    for name, N, Kd, act in (("c_attn", 3 * d, d, 0), ("c_fc", 4 * d, d, 1)):
        w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).to(dt)
        bias = torch.randn(N, device=dev).to(dt)
        cases.append((f"gemm_ln {name} +bias", lambda w=w, bias=bias, act=act: K.gemm_ln(x, lw, lb, 1e-5, w, bias, act=act)))
    for name, Kd in (("attn.c_proj", d), ("mlp.c_proj", 4 * d)):
        xa = torch.randn(B, Kd, device=dev).to(dt)
        w = (torch.randn(d, Kd, device=dev) / Kd ** 0.5).to(dt)
        bias = torch.randn(d, device=dev).to(dt)
        cases.append((f"gemm {name} +bias+res", lambda xa=xa, w=w, bias=bias: K.gemm(xa, w, bias, residual=res)))
    for name, fn in cases:
        ts = {"0": [], "1": []}
        outs = {}
        for _ in range(3):
            for pf in ("0", "1"):
                os.environ["MIFT_SKINNY_PF"] = pf
                ts[pf].append(timeit(fn))
                outs[pf] = fn()
        os.environ.pop("MIFT_SKINNY_PF")
        same = torch.equal(outs["0"][0] if isinstance(outs["0"], tuple) else outs["0"],
                           outs["1"][0] if isinstance(outs["1"], tuple) else outs["1"])
        row = {"name": name, "pf0_us": round(min(ts["0"]) * 1e3, 2), "pf1_us": round(min(ts["1"]) * 1e3, 2),
               "bit_identical": bool(same)}
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
