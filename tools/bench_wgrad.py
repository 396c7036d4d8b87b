"""Grouped LoRA weight-gradient launch at the distilgpt2 per-layer shapes (the 6 dB/dA problems of
one transformer layer in ONE lora_wgrad_group call), same-process interleaved A/B of env knobs.

  python tools/bench_wgrad.py "MIFT_WGRAD_BLOCKS=1024" "MIFT_WGRAD_BLOCKS=2048" [--p 0.05]
Also checks every arm against the first one (max |diff| of the accumulated arena).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mift.ops import kernels as K  # noqa: E402


def problems(M, dt, p, r=8):
    # (X columns, mode, dropout on X): c_attn dB (gz 2304) / dA (ln 768), attn.c_proj dB (768) / dA (768),
    # mlp.c_proj dB (768) / dA (gelu 3072)
    spec = [(2304, 1, 0.0), (768, 2, p), (768, 1, 0.0), (768, 2, p), (768, 1, 0.0), (3072, 2, p)]
    xs, ys, meta, ps, off = [], [], [], [], 0
    for i, (P, mode, pp) in enumerate(spec):
        xs.append(torch.randn(M, P, device="cuda", dtype=dt))
        y = torch.zeros(M, 32, device="cuda", dtype=dt)
        y[:, :r] = torch.randn(M, r, device="cuda", dtype=dt)
        ys.append(y)
        meta += [mode, 1, 0, r, off] + [0, 0, 0] * 3 + [1000 + i]
        ps.append(pp)
        off += P * r
    return xs, ys, meta, ps, off


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["X=0"])
    ap.add_argument("--p", type=float, default=0.05)
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    xs, ys, meta, ps, n = problems(a.M, torch.bfloat16, a.p)
    envs = [dict(kv.split("=", 1) for kv in c.split()) for c in a.configs]

    def run(env, out):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        K.lora_wgrad_group(out, xs, ys, meta, ps)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

    ref = None
    for c, env in zip(a.configs, envs):
        out = torch.zeros(n, device="cuda", dtype=torch.float32)
        run(env, out)
        torch.cuda.synchronize()
        if ref is None:
            ref = out
        else:
            d = (out - ref).abs().max().item()
            print(json.dumps({"config": c, "max_abs_diff_vs_first": d, "ref_max": ref.abs().max().item()}), flush=True)
    ts = {c: [] for c in a.configs}
    out = torch.zeros(n, device="cuda", dtype=torch.float32)
    for _ in range(a.rounds):
        for c, env in zip(a.configs, envs):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            s.record()
            for _ in range(a.iters):
                K.lora_wgrad_group(out, xs, ys, meta, ps)
            e.record()
            torch.cuda.synchronize()
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            ts[c].append(s.elapsed_time(e) / a.iters * 1000.0)
    mb = sum(x.numel() * 2 for x in xs) / 1e6
    for c in a.configs:
        us = statistics.median(ts[c])
        print(json.dumps({"config": c, "us": round(us, 2), "x_MB": round(mb, 1), "GBps": round(mb / us * 1e3, 0)}),
              flush=True)


if __name__ == "__main__":
    main()
