"""Epilogue cost of the OPT-2.7B block GEMMs on the phased 256x256 tile (fp16, M = 24576 = micro-batch
48 x 512): each GEMM plain, then with the epilogue features the training step adds one at a time
(bias, LoRA K-extension, activation / activation-backward on the stored auxiliary, residual dropout,
the next adapter's projection), to find which epilogue work the one-block-per-CU tile leaves exposed.

  python tools/bench_opt_epilogue.py [--M 24576] [--json out.json]
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
    ap.add_argument("--M", type=int, default=24576)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    mift._ext.require()
    dev, dt, M, D, F = "cuda", torch.float16, a.M, 2560, 10240
    torch.manual_seed(0)

    def rnd(*s, sc=1.0):
        return (torch.randn(*s, device=dev) * sc).to(dt)

    x = rnd(M, D)
    xf = rnd(M, F)
    res = rnd(M, D)
    a2 = rnd(M, 32, sc=0.1)
    out = []
    for name, A, N in (("qkv.fwd", x, 3 * D), ("out.fwd", x, D), ("fc1.fwd", x, F), ("fc2.fwd", xf, D),
                       ("fc2.dgrad", x, F), ("fc1.dgrad", xf, D)):
        Kd = A.shape[1]
        w = rnd(N, Kd, sc=0.02)
        bias = rnd(N, sc=0.02)
        b2 = rnd(N, 32, sc=0.1)
        pw = torch.zeros(32, N, device=dev, dtype=dt)
        pw[:16] = rnd(16, N, sc=0.02)
        aux = torch.relu(rnd(M, N)) if name == "fc2.dgrad" else None
        r = {"name": name, "M": M, "N": N, "K": Kd, "tflop": round(2 * M * N * Kd / 1e12, 3)}

        def t(**kw):
            return round(timeit(lambda: K.gemm(A, w, tile=8, **kw), iters=10, rounds=3) * 1e3, 1)

        r["plain"] = t()
        if name.endswith("fwd"):
            r["+bias"] = t(bias=bias)
            r["+bias+ext"] = t(bias=bias, a2=a2, b2=b2)
            if name == "fc1.fwd":
                r["+bias+ext+relu"] = t(bias=bias, a2=a2, b2=b2, act=2)
                r["+bias+ext+relu+proj"] = t(bias=bias, a2=a2, b2=b2, act=2, proj_w=pw, proj_rows=16,
                                             proj_p=0.05, proj_seed=5)
                bits = torch.empty(M, N // 8, dtype=torch.uint8, device=dev)
                r["+bias+ext+relu+proj+bits"] = t(bias=bias, a2=a2, b2=b2, act=2, proj_w=pw, proj_rows=16,
                                                  proj_p=0.05, proj_seed=5, sbits=bits)
            if name in ("out.fwd", "fc2.fwd"):
                r["+bias+ext+drop+res"] = t(bias=bias, a2=a2, b2=b2, residual=res, dropout_p=0.1, seed=3)
                os.environ["MIFT_EPI_PFG"] = "0"  # operands per chunk (the old rolled loop)
                r["+bias+ext+drop+res_pfg0"] = t(bias=bias, a2=a2, b2=b2, residual=res, dropout_p=0.1, seed=3)
                os.environ.pop("MIFT_EPI_PFG")
        else:
            r["+ext_masked"] = t(a2=a2, b2=b2, ext_p=0.05, ext_seed=3)
            if name == "fc2.dgrad":
                r["+ext_masked+relu_bwd"] = t(a2=a2, b2=b2, ext_p=0.05, ext_seed=3, act=5, aux=aux)
                r["+ext_masked+relu_bwd+proj"] = t(a2=a2, b2=b2, ext_p=0.05, ext_seed=3, act=5, aux=aux,
                                                   proj_w=pw, proj_rows=16, proj_alpha=2.0)
                bits = torch.empty(M, N // 8, dtype=torch.uint8, device=dev)
                K.gemm(A, w, act=2, sbits=bits, tile=8)  # sign bits of some ReLU output
                r["+ext_masked+relu_bwd_bits"] = t(a2=a2, b2=b2, ext_p=0.05, ext_seed=3, act=5, sbits=bits)
                r["+ext_masked+relu_bwd_bits+proj"] = t(a2=a2, b2=b2, ext_p=0.05, ext_seed=3, act=5, sbits=bits,
                                                        proj_w=pw, proj_rows=16, proj_alpha=2.0)
        if name == "fc2.dgrad":  # operands per chunk (the old rolled loop)
            os.environ["MIFT_EPI_PFG"] = "0"
            r["+ext_masked+relu_bwd_bits+proj_pfg0"] = t(a2=a2, b2=b2, ext_p=0.05, ext_seed=3, act=5, sbits=bits,
                                                         proj_w=pw, proj_rows=16, proj_alpha=2.0)
            r["+ext_masked+relu_bwd+proj_pfg0"] = t(a2=a2, b2=b2, ext_p=0.05, ext_seed=3, act=5, aux=aux,
                                                    proj_w=pw, proj_rows=16, proj_alpha=2.0)
            os.environ.pop("MIFT_EPI_PFG")
        r["plain_pf"] = round(r["tflop"] / r["plain"] * 1e3, 3)
        print(json.dumps(r), flush=True)
        out.append(r)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
