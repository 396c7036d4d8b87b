"""Wide-wave (4-wave, 128x128 per wave) 256x256 kernels vs the phased 8-wave ones.

  python tools/bench_wide.py [--json out.jsonl]

For the fused LM head (forward: E / stats / loss; dgrad: dX) at distilgpt2 and OPT-2.7B shapes and
for plain gemm_nt at large shapes: checks the two schedules agree (forward bit-identical: the same
MFMA order per accumulator; dgrad within fp32 reassociation), then times both (CUDA events,
interleaved rounds in one process, random data) plus torch.matmul (hipBLASLt) for reference.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mift.ops import kernels as K  # noqa: E402


def timeit(fn, iters=10, rounds=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1000 / iters)
    return round(statistics.median(ts), 1)


def lmhead_case(name, M, d, V, dtype):
    Vp = (V + 255) // 256 * 256 if False else (V + 63) // 64 * 64
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, d, device="cuda", dtype=dtype, generator=g)
    W = torch.zeros(Vp, d, device="cuda", dtype=dtype)
    W[:V] = (0.05 * torch.randn(V, d, device="cuda", generator=g)).to(dtype)
    Wt = W.t().contiguous()
    lab = torch.randint(0, V, (M,), device="cuda", generator=g)
    gs = torch.full((1,), 1.0 / M, device="cuda")
    out = {}
    res = {}
    for wide in ("0", "1"):
        os.environ["MIFT_LM_WIDE"] = wide
        E, st, lse, loss, zl = K.lmhead_fwd(x, W, lab, V)
        dx = K.lmhead_dgrad(E, Wt, W, lab, V, st, lse, gs)
        res[wide] = (E, st, lse, loss, dx)
        out[f"fwd_w{wide}_us"] = timeit(lambda: K.lmhead_fwd(x, W, lab, V))
        out[f"dgrad_w{wide}_us"] = timeit(lambda: K.lmhead_dgrad(E, Wt, W, lab, V, st, lse, gs))
    os.environ.pop("MIFT_LM_WIDE", None)
    a, b = res["0"], res["1"]
    out["E_equal"] = bool(torch.equal(a[0], b[0]))
    out["loss_maxdiff"] = float((a[3] - b[3]).abs().max())
    out["dx_rel"] = float((a[4].float() - b[4].float()).norm() / a[4].float().norm())
    # fp32 reference of the loss / dX on a row subset
    r = slice(0, 256)
    z = x[r].float() @ W[:V].float().t()
    ref_loss = torch.nn.functional.cross_entropy(z, lab[r], reduction="none")
    out["loss_vs_fp32"] = float((b[3][r] - ref_loss).abs().max())
    p = torch.softmax(z, -1)
    p[torch.arange(256, device="cuda"), lab[r]] -= 1
    ref_dx = (p @ W[:V].float()) / M
    out["dx_vs_fp32_rel"] = float((b[4][r].float() - ref_dx).norm() / ref_dx.norm())
    out["blas_fwd_us"] = timeit(lambda: x @ W.t())
    fl = 2.0 * M * Vp * d
    out["fwd_w1_TF"] = round(fl / out["fwd_w1_us"] / 1e6, 1)
    out["dgrad_w1_TF"] = round(fl / out["dgrad_w1_us"] / 1e6, 1)
    return dict(name=name, M=M, d=d, V=V, **out)


def gemm_case(name, M, N, Kd, dtype):
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.randn(M, Kd, device="cuda", dtype=dtype, generator=g)
    b = (0.05 * torch.randn(N, Kd, device="cuda", generator=g)).to(dtype)
    out = {}
    y8 = K.gemm(a, b, tile=8)
    y10 = K.gemm(a, b, tile=10)
    ref = (a[:512].float() @ b.float().t())
    out["t10_vs_fp32_rel"] = float((y10[:512].float() - ref).norm() / ref.norm())
    out["t8_t10_equal"] = bool(torch.equal(y8, y10))
    for t in (8, 10):
        out[f"t{t}_us"] = timeit(lambda: K.gemm(a, b, tile=t))
    out["blas_us"] = timeit(lambda: a @ b.t())
    out["t10_TF"] = round(2.0 * M * N * Kd / out["t10_us"] / 1e6, 1)
    return dict(name=name, M=M, N=N, K=Kd, **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    rows = []
    cases = [("lm.distilgpt2", lambda: lmhead_case("lm.distilgpt2", 8192, 768, 50257, torch.bfloat16)),
             ("lm.opt27b.mb8", lambda: lmhead_case("lm.opt27b.mb8", 4096, 2560, 50272, torch.float16)),
             ("gemm.opt.fc1", lambda: gemm_case("gemm.opt.fc1", 24576, 10240, 2560, torch.float16)),
             ("gemm.square4k", lambda: gemm_case("gemm.square4k", 4096, 4096, 4096, torch.bfloat16))]
    for name, fn in cases:
        if a.only and a.only not in name:
            continue
        r = fn()
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
