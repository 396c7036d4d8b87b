"""Column-split of the wide distilgpt2 GEMMs (N = 2304 / 3072, K = 768): the phased 256x256 tile
(tile 8) on the first 2048 columns — 256 tiles, exactly one per CU — plus a second launch for the
remaining columns, against the auto tile over the whole N (128x192 at 1.5-2 tile rounds per CU slot).
Epilogues as in the step (bias + LoRA K-extension; GELU + pre-activation store; GELU backward on
the stored pre-activation + dropout-masked extension).

  python tools/bench_split_n.py [--json out.json]
"""
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
    ap.add_argument("--rest", default="6,3,7,4,9")
    a = ap.parse_args()
    mift._ext.require()
    dev, dt, M, Kd = "cuda", torch.bfloat16, 8192, 768
    torch.manual_seed(0)
    x = torch.randn(M, Kd, device=dev).to(dt)
    a2 = (torch.randn(M, 32, device=dev) * 0.1).to(dt)
    out = []
    for name, N in (("c_attn.fwd", 2304), ("mlp.c_fc.fwd", 3072), ("mlp.c_proj.dgrad", 3072)):
        w = (torch.randn(N, Kd, device=dev) * 0.02).to(dt)
        bias = (torch.randn(N, device=dev) * 0.02).to(dt)
        b2 = (torch.randn(N, 32, device=dev) * 0.1).to(dt)
        aux = torch.randn(M, N, device=dev).to(dt)

        sl = {(c0, c1): (w[c0:c1], bias[c0:c1], b2[c0:c1].contiguous(), aux[:, c0:c1].contiguous())
              for c0, c1 in ((0, N), (0, 2048), (2048, N))}

        def call(c0, c1, tile):
            ws, bs, b2s, auxs = sl[(c0, c1)]
            if name == "c_attn.fwd":
                return K.gemm(x, ws, bs, a2, b2s, tile=tile)
            if name == "mlp.c_fc.fwd":
                return K.gemm(x, ws, bs, act=1, want_preact=True, tile=tile)
            return K.gemm(x, ws, None, a2, b2s, act=4, aux=auxs, ext_p=0.05, ext_seed=3, tile=tile)

        r = {"name": name, "M": M, "N": N, "K": Kd}
        r["auto_us"] = round(timeit(lambda: call(0, N, 0)) * 1e3, 1)
        r["t8_full_us"] = round(timeit(lambda: call(0, N, 8)) * 1e3, 1)
        r["t8_2048_us"] = round(timeit(lambda: call(0, 2048, 8)) * 1e3, 1)
        for t in [int(v) for v in a.rest.split(",")]:
            r[f"rest_t{t}_us"] = round(timeit(lambda: call(2048, N, t)) * 1e3, 1)
            r[f"split_t8+t{t}_us"] = round(timeit(lambda: (call(0, 2048, 8), call(2048, N, t))) * 1e3, 1)
        print(json.dumps(r), flush=True)
        out.append(r)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
