"""LN backward + residual-dropout backward + dT projection: one pass (rowproj MODE 3) vs ln_bwd8 then
mask_proj, at the distilgpt2 shape (M = 8192, D = 768, rank 8, p = 0.1).

  python tools/bench_ln_mask_proj.py [--json out.json]"""
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
    M, D, dt = 8192, 768, torch.bfloat16
    torch.manual_seed(0)
    x = torch.randn(M, D, device="cuda").to(dt)
    dy = torch.randn(M, D, device="cuda").to(dt)
    gr = torch.randn(M, D, device="cuda").to(dt)
    w = torch.ones(D, device="cuda", dtype=dt)
    _, mean, rstd = K.layer_norm_fwd(x, w, torch.zeros_like(w), 1e-5)
    pw = torch.zeros(32, D, device="cuda", dtype=dt)
    pw[:8] = (torch.randn(8, D, device="cuda") / D ** 0.5).to(dt)
    fused = lambda: K.ln_bwd_mask_proj(dy, x, w, mean, rstd, gr, 0.1, 5, pw, 8, 2.0)  # noqa: E731
    sep = lambda: K.mask_proj(K.layer_norm_bwd(dy, x, w, mean, rstd, dres=gr)[0], 0.1, 5, pw, 8, 2.0)  # noqa: E731
    lnb = lambda: K.layer_norm_bwd(dy, x, w, mean, rstd, dres=gr)  # noqa: E731
    rows = []
    for name, fn in (("ln_bwd_mask_proj (one pass)", fused), ("layer_norm_bwd + mask_proj", sep), ("layer_norm_bwd alone", lnb)):
        row = {"name": name, "us": round(min(timeit(fn) for _ in range(3)) * 1e3, 2)}
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
