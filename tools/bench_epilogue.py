"""Cost of each fused GEMM epilogue stage at the distilgpt2 MLP shapes (M=8192, N=3072, K=768).

  python tools/bench_epilogue.py
Variants: plain, +bias, +gelu (+preact store), +gelu-bwd (aux read), +masked LoRA ext, full fc2-dgrad.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mift  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    C = mift._ext.require()
    M, N, K = 8192, 3072, 768
    dt = torch.bfloat16
    a = torch.randn(M, K, device="cuda", dtype=dt)
    b = torch.randn(N, K, device="cuda", dtype=dt) / K ** 0.5
    bias = torch.randn(N, device="cuda", dtype=dt)
    aux = torch.randn(M, N, device="cuda", dtype=dt)
    a2 = torch.randn(M, 32, device="cuda", dtype=dt)
    b2 = torch.randn(N, 32, device="cuda", dtype=dt)
    fl = 2.0 * M * N * K

    def g(**kw):
        args = dict(bias=None, a2=None, b2=None, act=0, aux=None, residual=None, p=0.0, seed=0, pre=False,
                    ext_p=0.0, tile=int(os.environ.get("TILE", "0")))
        args.update(kw)
        return lambda: C.gemm_nt(a, b, args["bias"], args["a2"], args["b2"], args["act"], args["aux"],
                                 args["residual"], args["p"], args["seed"], args["pre"], 1.0, None, args["tile"],
                                 None, None, args["ext_p"], 7)

    variants = [
        ("plain", g()),
        ("bias", g(bias=bias)),
        ("bias+gelu", g(bias=bias, act=1)),
        ("bias+gelu+preact (fc1 fwd)", g(bias=bias, act=1, pre=True)),
        ("gelu_bwd(aux)", g(act=4, aux=aux)),
        ("ext", g(a2=a2, b2=b2)),
        ("ext masked", g(a2=a2, b2=b2, ext_p=0.05)),
        ("ext masked + gelu_bwd (fc2 dgrad)", g(a2=a2, b2=b2, ext_p=0.05, act=4, aux=aux)),
        ("dropout 0.1 epilogue", g(p=0.1, seed=3)),
    ]
    for name, fn in variants:
        t = timeit(fn)
        print(f"{name:36s} {t * 1e3:8.1f} us  {fl / t / 1e9:7.1f} TF/s", flush=True)
    t = timeit(lambda: torch.matmul(a, b.t()))
    print(f"{'torch.matmul (hipBLASLt)':36s} {t * 1e3:8.1f} us  {fl / t / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
