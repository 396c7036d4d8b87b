"""LM head + CE per-step cost at distilgpt2 / OPT shapes: fused HIP head vs the hipBLASLt path.

Times forward + backward of ops.fused.lm_head_xent (LN, head GEMMs, CE) with CUDA events,
interleaved rounds in one process (guide rule 24), random data.
  python tools/bench_lmhead.py [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mift.ops import fused as F  # noqa: E402


class _LN(torch.nn.Module):
    def __init__(self, d, dtype):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.ones(d, device="cuda", dtype=dtype), requires_grad=False)
        self.bias = torch.nn.Parameter(torch.zeros(d, device="cuda", dtype=dtype), requires_grad=False)
        self.eps = 1e-5


def run(M, d, V, dtype, iters=10, rounds=5):
    Vp = (V + 63) // 64 * 64
    h = torch.randn(M, d, device="cuda", dtype=dtype, requires_grad=True)
    W = torch.zeros(Vp, d, device="cuda", dtype=dtype)
    W[:V] = 0.02 * torch.randn(V, d, device="cuda", dtype=dtype)
    Wt = W.t().contiguous()
    lab = torch.randint(0, V, (M,), device="cuda")
    ln = _LN(d, dtype)

    def step(mode):
        os.environ["MIFT_LMHEAD"] = mode
        loss = F.lm_head_xent(h, ln, W, lab, V, -100, need_grad=True, w_kn=Wt)
        loss.backward()
        h.grad = None

    res = {}
    for mode in ("fused", "blas"):
        step(mode)
    torch.cuda.synchronize()
    ts = {"fused": [], "blas": []}
    for _ in range(rounds):
        for mode in ("fused", "blas"):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                step(mode)
            e.record()
            torch.cuda.synchronize()
            ts[mode].append(s.elapsed_time(e) / iters)
    for mode in ts:
        res[mode + "_ms"] = round(statistics.median(ts[mode]), 4)
    os.environ.pop("MIFT_LMHEAD", None)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = []
    for name, M, d, V, dt in [("distilgpt2", 8192, 768, 50257, torch.bfloat16),
                              ("opt-2.7b.mb8", 4096, 2560, 50272, torch.float16)]:
        r = dict(name=name, M=M, d=d, V=V, **run(M, d, V, dt))
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
