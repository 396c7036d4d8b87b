"""Micro-benchmarks of the mift HIP kernels vs the torch/hipBLASLt equivalent.

Usage:  python tools/bench_kernels.py [--only gemm,ln,attn,xent] [--json out.json]
Timing: CUDA events around `iters` back-to-back launches after warmup, on
random data (guide §5.4 rule 25), median of 5 rounds, both variants
interleaved in one process (rule 24).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import mift  # noqa: E402


def timeit(fn, iters=20, rounds=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters)
    return statistics.median(ts)


TILES = [int(t) for t in os.environ.get("TILES", "0,1,2,3,4,5,6,7").split(",")]
GEMM_SHAPES = [
    # (name, M, N, K)  distilgpt2, 32x256 tokens per rank
    ("c_attn.fwd", 8192, 2304, 768),
    ("attn.c_proj.fwd", 8192, 768, 768),
    ("mlp.c_fc.fwd", 8192, 3072, 768),
    ("mlp.c_proj.fwd", 8192, 768, 3072),
    ("c_attn.dgrad", 8192, 768, 2304),
    ("mlp.c_fc.dgrad", 8192, 768, 3072),
    ("mlp.c_proj.dgrad", 8192, 3072, 768),
    ("lm_head.fwd", 8192, 50304, 768),
    ("lm_head.dgrad", 8192, 768, 50304),
    ("square4k", 4096, 4096, 4096),
]
OPT_SHAPES = [  # OPT-2.7B, 8x512 tokens per micro-batch (every distinct GEMM of a layer)
    ("opt.qkv.fwd", 4096, 7680, 2560), ("opt.out.fwd", 4096, 2560, 2560), ("opt.fc1.fwd", 4096, 10240, 2560),
    ("opt.fc2.fwd", 4096, 2560, 10240), ("opt.qkv.dgrad", 4096, 2560, 7680), ("opt.fc1.dgrad", 4096, 2560, 10240),
    ("opt.fc2.dgrad", 4096, 10240, 2560), ("opt.lm_head.fwd", 4096, 50304, 2560),
    ("opt.fc2.fwd.M2k", 2048, 2560, 10240), ("opt.fc2.fwd.M16k", 16384, 2560, 10240),
]


# the eight distinct GEMMs of an OPT-2.7B layer (forward + dgrad), N x K at M = micro-batch x 512
OPT_LAYER = [("opt.qkv.fwd", 7680, 2560), ("opt.out.fwd", 2560, 2560), ("opt.fc1.fwd", 10240, 2560),
             ("opt.fc2.fwd", 2560, 10240), ("opt.qkv.dgrad", 2560, 7680), ("opt.out.dgrad", 2560, 2560),
             ("opt.fc1.dgrad", 2560, 10240), ("opt.fc2.dgrad", 10240, 2560)]


def bench_gemm(results, shapes=None, dtype=torch.bfloat16):
    import mift._C as C
    for name, M, N, K in shapes or GEMM_SHAPES:
        a = torch.randn(M, K, device="cuda", dtype=dtype)
        b = torch.randn(N, K, device="cuda", dtype=dtype)
        fl = 2.0 * M * N * K
        row = {"name": name, "M": M, "N": N, "K": K}
        for tile in TILES:
            t = timeit(lambda: C.gemm_nt(a, b, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, tile, None, None, 0.0, 0))
            row[f"mift_t{tile}_ms"] = round(t, 4)
            row[f"mift_t{tile}_tflops"] = round(fl / t / 1e9, 1)
        t = timeit(lambda: torch.matmul(a, b.t()))
        row["torch_ms"] = round(t, 4)
        row["torch_tflops"] = round(fl / t / 1e9, 1)
        print(json.dumps(row), flush=True)
        results.append(row)


# distilgpt2 GEMMs with the epilogues they run with in training (fused block Functions)
DGPT_CASES = [
    # name, M, N, K, epilogue kwargs
    ("c_attn.fwd+ext+bias", 8192, 2304, 768, dict(bias=1, ext=1)),
    ("attn.c_proj.fwd+ext+drop+res", 8192, 768, 768, dict(bias=1, ext=1, p=0.1, res=1)),
    ("c_fc.fwd+gelu+preact", 8192, 3072, 768, dict(bias=1, act=1, pre=1)),
    ("mlp.c_proj.fwd+ext+drop+res", 8192, 768, 3072, dict(bias=1, ext=1, p=0.1, res=1)),
    ("c_attn.dgrad+maskext", 8192, 768, 2304, dict(ext=1, ext_p=0.05)),
    ("c_fc.dgrad", 8192, 768, 3072, dict()),
    ("mlp.c_proj.dgrad+maskext+gelubwd", 8192, 3072, 768, dict(ext=1, ext_p=0.05, act=4, aux=1)),
    ("attn.c_proj.dgrad+maskext", 8192, 768, 768, dict(ext=1, ext_p=0.05)),
]


OPT_CASES = [  # OPT-2.7B at micro-batch 48 x 512 tokens, fp16
    ("opt.out.fwd+ext+drop+res", 24576, 2560, 2560, dict(bias=1, ext=1, p=0.1, res=1)),
    ("opt.fc1.fwd+ext+relu", 24576, 10240, 2560, dict(bias=1, ext=1, act=2)),
    ("opt.fc2.fwd+ext+drop+res", 24576, 2560, 10240, dict(bias=1, ext=1, p=0.1, res=1)),
    ("opt.fc2.dgrad+maskext+relubwd", 24576, 10240, 2560, dict(ext=1, ext_p=0.05, act=5, aux=1)),
    ("opt.qkv.dgrad+maskext", 24576, 2560, 7680, dict(ext=1, ext_p=0.05)),
]


def bench_epi_ab(results):
    """Epilogue form A/B (MIFT_EPI_STAGED 0 = per-chunk, 1 = feature-staged) interleaved in one process
    (guide rule 24)."""
    import mift._C as C
    for name, M, N, K, e in DGPT_CASES + OPT_CASES:
        dt = torch.float16 if name.startswith("opt") else torch.bfloat16
        a = torch.randn(M, K, device="cuda", dtype=dt)
        b = torch.randn(N, K, device="cuda", dtype=dt) / K ** 0.5
        bias = torch.randn(N, device="cuda", dtype=dt) if e.get("bias") else None
        a2 = torch.randn(M, 32, device="cuda", dtype=dt) if e.get("ext") else None
        b2 = torch.randn(N, 32, device="cuda", dtype=dt) if e.get("ext") else None
        aux = torch.randn(M, N, device="cuda", dtype=dt) if e.get("aux") else None
        res = torch.randn(M, N, device="cuda", dtype=dt) if e.get("res") else None
        fn = lambda: C.gemm_nt(a, b, bias, a2, b2, e.get("act", 0), aux, res, e.get("p", 0.0), 3,  # noqa: E731
                               bool(e.get("pre", 0)), 1.0, None, 0, None, None, e.get("ext_p", 0.0), 7)
        ts = {0: [], 1: []}
        for _ in range(3):
            for pf in (0, 1):
                os.environ["MIFT_EPI_STAGED"] = str(pf)
                ts[pf].append(timeit(fn, rounds=3))
        os.environ.pop("MIFT_EPI_STAGED", None)
        row = {"name": name, "per_chunk_us": round(min(ts[0]) * 1e3, 1), "staged_us": round(min(ts[1]) * 1e3, 1)}
        print(json.dumps(row), flush=True)
        results.append(row)


def opt_m_cases(Ms=(2048, 4096, 24576)):
    """OPT-2.7B layer GEMMs (with their training epilogues) at the micro-batch sizes of the PP configs:
    M = mb x 512 tokens (mb 4 / 8 / 48)."""
    base = [("opt.qkv.fwd+ext+bias", 7680, 2560, dict(bias=1, ext=1)),
            ("opt.out.fwd+ext+drop+res", 2560, 2560, dict(bias=1, ext=1, p=0.1, res=1)),
            ("opt.fc1.fwd+ext+relu", 10240, 2560, dict(bias=1, ext=1, act=2)),
            ("opt.fc2.fwd+ext+drop+res", 2560, 10240, dict(bias=1, ext=1, p=0.1, res=1)),
            ("opt.fc2.dgrad+maskext+relubwd", 10240, 2560, dict(ext=1, ext_p=0.05, act=5, aux=1)),
            ("opt.fc1.dgrad+maskext", 2560, 10240, dict(ext=1, ext_p=0.05)),
            ("opt.out.dgrad+maskext", 2560, 2560, dict(ext=1, ext_p=0.05)),
            ("opt.qkv.dgrad+maskext", 2560, 7680, dict(ext=1, ext_p=0.05))]
    return [(f"{n}@M{M}", M, N, K, e) for M in Ms for n, N, K, e in base]


def bench_dgpt(results, cases=None, dt=torch.bfloat16):
    import mift._C as C
    tot = {}
    for name, M, N, K, e in cases or DGPT_CASES:
        a = torch.randn(M, K, device="cuda", dtype=dt)
        b = torch.randn(N, K, device="cuda", dtype=dt) / K ** 0.5
        bias = torch.randn(N, device="cuda", dtype=dt) if e.get("bias") else None
        a2 = torch.randn(M, 32, device="cuda", dtype=dt) if e.get("ext") else None
        b2 = torch.randn(N, 32, device="cuda", dtype=dt) if e.get("ext") else None
        aux = torch.randn(M, N, device="cuda", dtype=dt) if e.get("aux") else None
        res = torch.randn(M, N, device="cuda", dtype=dt) if e.get("res") else None
        fl = 2.0 * M * N * K
        row = {"name": name, "M": M, "N": N, "K": K}
        for tile in TILES:
            t = timeit(lambda: C.gemm_nt(a, b, bias, a2, b2, e.get("act", 0), aux, res, e.get("p", 0.0), 3,
                                         bool(e.get("pre", 0)), 1.0, None, tile, None, None, e.get("ext_p", 0.0), 7))
            row[f"mift_t{tile}_us"] = round(t * 1e3, 1)
            row[f"mift_t{tile}_tflops"] = round(fl / t / 1e9, 1)
            tot[tile] = tot.get(tile, 0.0) + t * 1e3
        print(json.dumps(row), flush=True)
        results.append(row)
    print("per-layer total us by tile:", json.dumps({k: round(v, 1) for k, v in tot.items()}), flush=True)
    return tot


def bench_ln(results):
    import mift._C as C
    for M, D in [(8192, 768), (2048, 2560), (8192, 4096)]:
        x = torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
        w = torch.ones(D, device="cuda", dtype=torch.bfloat16)
        b = torch.zeros(D, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: C.layer_norm_fwd(x, w, b, 1e-5))
        tt = timeit(lambda: torch.nn.functional.layer_norm(x, (D,), w, b, 1e-5))
        gbs = 2 * x.numel() * 2 / t / 1e6
        row = {"name": f"ln_fwd_{M}x{D}", "mift_ms": round(t, 4), "mift_GBps": round(gbs, 1),
               "torch_ms": round(tt, 4)}
        print(json.dumps(row), flush=True)
        results.append(row)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="gemm,ln")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    assert mift.kernels_available(), mift._ext.error()
    results = []
    for k in a.only.split(","):
        {"gemm": bench_gemm, "ln": bench_ln, "dgpt": bench_dgpt, "epi": bench_epi_ab,
         "opt": lambda r: bench_gemm(r, OPT_SHAPES, torch.float16),
         # vs hipBLASLt (torch.matmul) at micro-batch 12 and 48: TILES=0 for auto only
         "opt_blas": lambda r: bench_gemm(r, [(f"{n}@M{M}", M, N, K) for M in (6144, 24576)
                                              for n, N, K in OPT_LAYER], torch.float16),
         "optm": lambda r: bench_dgpt(r, opt_m_cases(), torch.float16),
         "optm_small": lambda r: bench_dgpt(r, opt_m_cases((2048, 4096)), torch.float16),
         "optm_pp": lambda r: bench_dgpt(r, opt_m_cases((2048, 6144)), torch.float16)}[k](results)
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
