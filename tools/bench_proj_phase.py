"""The GEMM projection-phase cost at OPT's fc1 shape (M = 24576, N = 10240, K = 2560, fp16, ReLU): the
epilogue with / without the projection, with / without its LoRA-input dropout hash, 16 vs 32 rows.
Run under rocprofv3 --kernel-trace to split the GEMM from proj_reduce.

  python tools/bench_proj_phase.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import mift  # noqa: E402
from mift.ops import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    mift._ext.require()
    dev, dt, M, N, Kd = "cuda", torch.float16, 24576, 10240, 2560
    torch.manual_seed(0)
    x = torch.randn(M, Kd, device=dev).to(dt)
    w = (torch.randn(N, Kd, device=dev) * 0.02).to(dt)
    bias = (torch.randn(N, device=dev) * 0.02).to(dt)
    pw = torch.zeros(32, N, device=dev, dtype=dt)
    pw[:32] = (torch.randn(32, N, device=dev) * 0.02).to(dt)
    r = {}

    def t(**kw):
        return round(timeit(lambda: K.gemm(x, w, bias, act=2, tile=8, **kw), iters=10, rounds=3) * 1e3, 1)

    r["relu"] = t()
    r["relu+proj16_p0"] = t(proj_w=pw, proj_rows=16)
    r["relu+proj16_p05"] = t(proj_w=pw, proj_rows=16, proj_p=0.05, proj_seed=5)
    r["relu+proj32_p0"] = t(proj_w=pw, proj_rows=32)
    r["relu+proj8_p0"] = t(proj_w=pw, proj_rows=8)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
