"""The 4-wave 256x256 GEMM schedule (tile 10, gemm.hip mainloop4) against the phased 8-wave loop
(tile 8) and hipBLASLt (torch.matmul).

  python tools/bench_gemm4.py [--check-only] [--json out.json] [--tiles 8,10]

1. Numerics: tile 10 must equal tile 8 bit for bit (same per-element MFMA accumulation order, same
   epilogue) on ragged shapes, 1-3 k-tiles and the training epilogues, and both are compared with an
   fp32 reference of the plain product.
2. Timing (guide §5.4 rules 24/25): random operands, every variant interleaved in one process, median
   of 5 rounds: the 16 OPT-2.7B layer (M, shape) pairs of VERDICT r5 item 1, the distilgpt2 LM-head
   shapes and square 4096^3.
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


def gemm(C, a, b, tile, e=None, aux=None, res=None, bias=None, a2=None, b2=None):
    e = e or {}
    return C.gemm_nt(a, b, bias, a2, b2, e.get("act", 0), aux, res, e.get("p", 0.0), 3, bool(e.get("pre", 0)),
                     1.0, None, tile, None, None, e.get("ext_p", 0.0), 7)[0]


def operands(M, N, K, dt, e=None, scale=True):
    e = e or {}
    a = torch.randn(M, K, device="cuda", dtype=dt)
    b = torch.randn(N, K, device="cuda", dtype=dt)
    if scale:
        b = b / K ** 0.5
    ops = dict(
        bias=torch.randn(N, device="cuda", dtype=dt) if e.get("bias") else None,
        a2=torch.randn(M, 32, device="cuda", dtype=dt) if e.get("ext") else None,
        b2=torch.randn(N, 32, device="cuda", dtype=dt) if e.get("ext") else None,
        aux=torch.randn(M, N, device="cuda", dtype=dt) if e.get("aux") else None,
        res=torch.randn(M, N, device="cuda", dtype=dt) if e.get("res") else None)
    return a, b, ops


CHECKS = [  # (M, N, K, dtype, epilogue)
    (256, 256, 64, torch.bfloat16, {}), (256, 256, 128, torch.float16, {}), (256, 256, 192, torch.bfloat16, {}),
    (1000, 704, 640, torch.bfloat16, {}), (513, 264, 2560, torch.float16, {}), (4096, 4096, 4096, torch.bfloat16, {}),
    (2048, 2560, 2560, torch.float16, dict(bias=1, ext=1, p=0.1, res=1)),
    (2048, 10240, 2560, torch.float16, dict(bias=1, ext=1, act=2)),
    (2048, 10240, 2560, torch.float16, dict(ext=1, ext_p=0.05, act=5, aux=1)),
    (1536, 3072, 768, torch.bfloat16, dict(bias=1, act=1, pre=1)),
    (777, 2304, 704, torch.bfloat16, dict(bias=1, ext=1)),
]

OPT_LAYER = [("opt.qkv.fwd", 7680, 2560), ("opt.out.fwd", 2560, 2560), ("opt.fc1.fwd", 10240, 2560),
             ("opt.fc2.fwd", 2560, 10240), ("opt.qkv.dgrad", 2560, 7680), ("opt.out.dgrad", 2560, 2560),
             ("opt.fc1.dgrad", 2560, 10240), ("opt.fc2.dgrad", 10240, 2560)]


def check(C, tiles):
    ok = True
    for M, N, K, dt, e in CHECKS:
        a, b, o = operands(M, N, K, dt, e)
        outs = {t: gemm(C, a, b, t, e, **o) for t in tiles}
        torch.cuda.synchronize()
        row = {"check": f"{M}x{N}x{K}", "dtype": str(dt).split(".")[-1], "epi": e}
        ref = outs[tiles[0]]
        for t in tiles[1:]:
            row[f"t{t}_eq_t{tiles[0]}"] = bool(torch.equal(outs[t], ref))
            row[f"t{t}_maxdiff"] = float((outs[t].float() - ref.float()).abs().max())
            ok = ok and row[f"t{t}_eq_t{tiles[0]}"]
        if not e:
            r = a.float() @ b.float().t()
            for t in tiles:
                row[f"t{t}_rel_fp32"] = float((outs[t].float() - r).norm() / r.norm())
                ok = ok and row[f"t{t}_rel_fp32"] < 1e-2
        print(json.dumps(row), flush=True)
    return ok


def bench(C, tiles, results, only=None):
    shapes = [(f"{n}@M{M}", M, N, K, torch.float16) for M in (6144, 24576) for n, N, K in OPT_LAYER]
    shapes += [("lm_head.fwd.dgpt", 8192, 50304, 768, torch.bfloat16),
               ("lm_head.dgrad.dgpt", 8192, 768, 50304, torch.bfloat16),
               ("square4k", 4096, 4096, 4096, torch.bfloat16),
               ("opt.lm_head.fwd@M6144", 6144, 50304, 2560, torch.float16),
               # split-K proxy of the LM-head dgrad: its 8 K-chunks of 6288 as 8x the rows (same tiles,
               # same per-tile K length, same FLOPs; no partial-slab reduction)
               ("lm_head.dgrad.dgpt.split8_proxy", 8 * 8192, 768, 6272, torch.bfloat16)]
    if only:
        shapes = [s for s in shapes if any(o in s[0] for o in only.split(","))]
    wins = 0
    for name, M, N, K, dt in shapes:
        a, b, _ = operands(M, N, K, dt, scale=False)
        fl = 2.0 * M * N * K
        row = {"name": name, "M": M, "N": N, "K": K}
        fns = {f"t{t}": (lambda t=t: gemm(C, a, b, t)) for t in tiles}
        fns["blas"] = lambda: torch.matmul(a, b.t())
        ts = {k: [] for k in fns}
        for _ in range(3):  # interleaved rounds (rule 24)
            for k, f in fns.items():
                ts[k].append(timeit(f, rounds=3))
        for k in fns:
            t = min(ts[k])
            row[f"{k}_us"] = round(t * 1e3, 1)
            row[f"{k}_TF"] = round(fl / t / 1e9, 1)
        if "t10" in fns:
            row["t10_vs_blas"] = round(row["blas_us"] / row["t10_us"], 3)
            wins += row["t10_vs_blas"] >= 1.0
        print(json.dumps(row), flush=True)
        results.append(row)
    print(json.dumps({"t10_ge_blas": wins, "of": len(shapes)}), flush=True)


def sweep(C, tiles, results):
    """K sweep at one chip round of tiles (M = 6144, N = 2560: 240 256x256 tiles): time = per-tile
    overhead (prologue, epilogue) + K/64 x per-k-tile main-loop time, separated by a linear fit."""
    for M, N in ((6144, 2560), (4096, 4096)):
        pts = {}
        for K in (640, 1280, 2560, 5120, 10240):
            a, b, _ = operands(M, N, K, torch.float16, scale=False)
            fns = {f"t{t}": (lambda t=t: gemm(C, a, b, t)) for t in tiles}
            fns["blas"] = lambda: torch.matmul(a, b.t())
            ts = {k: [] for k in fns}
            for _ in range(3):
                for k, f in fns.items():
                    ts[k].append(timeit(f, rounds=3))
            row = {"sweep": f"{M}x{N}", "K": K}
            for k in fns:
                row[f"{k}_us"] = round(min(ts[k]) * 1e3, 1)
                pts.setdefault(k, []).append((K / 64, min(ts[k]) * 1e3))
            print(json.dumps(row), flush=True)
            results.append(row)
        for k, xy in pts.items():
            n = len(xy)
            mx = sum(x for x, _ in xy) / n
            my = sum(y for _, y in xy) / n
            slope = sum((x - mx) * (y - my) for x, y in xy) / sum((x - mx) ** 2 for x, _ in xy)
            fit = {"fit": f"{M}x{N}", "variant": k, "us_per_ktile": round(slope, 3), "overhead_us": round(my - slope * mx, 1)}
            print(json.dumps(fit), flush=True)
            results.append(fit)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--tiles", default="8,10")
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="comma-separated name filters for the timing shapes")
    a = ap.parse_args()
    assert mift.kernels_available(), mift._ext.error()
    import mift._C as C
    tiles = [int(t) for t in a.tiles.split(",")]
    ok = check(C, tiles)
    print(json.dumps({"checks_ok": ok}), flush=True)
    if a.check_only or not ok:
        sys.exit(0 if ok else 1)
    results = []
    if a.sweep:
        sweep(C, tiles, results)
    else:
        bench(C, tiles, results, a.only)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
