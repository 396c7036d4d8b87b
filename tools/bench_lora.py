"""LoRA side-path kernels at distilgpt2-step shapes: same-process interleaved A/B of the
env-switchable launch choices (MIFT_LORA_MT for lora_proj, MIFT_WGRAD_BLOCKS for lora_wgrad).

Whole-process bench.py A/B on one box varies by ~10% run to run; kernel choices are decided here
instead (CUDA events, interleaved rounds, medians — guide rule 24).
  python tools/bench_lora.py [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mift.ops import kernels as K  # noqa: E402


def timed(fn, variants, envkey, iters=20, rounds=7):
    for v in variants:
        os.environ[envkey] = str(v)
        fn()
    torch.cuda.synchronize()
    ts = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            os.environ[envkey] = str(v)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            ts[v].append(s.elapsed_time(e) / iters * 1000.0)
    os.environ.pop(envkey, None)
    return {f"{envkey}={v}": round(statistics.median(ts[v]), 2) for v in variants}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--M", type=int, default=8192)
    a = ap.parse_args()
    M, dt = a.M, torch.bfloat16
    rows = []
    for Kd in (768, 3072):
        x = torch.randn(M, Kd, device="cuda", dtype=dt)
        w32 = torch.zeros(32, Kd, device="cuda", dtype=dt)
        w32[:8] = 0.02 * torch.randn(8, Kd, device="cuda", dtype=dt)
        r = {"op": "lora_proj", "M": M, "K": Kd, "us": timed(lambda: K.lora_proj(x, w32, 2.0, 0.05, 7, 8),
                                                                 (1, 2), "MIFT_LORA_MT")}
        print(json.dumps(r), flush=True)
        rows.append(r)
    for P in (768, 2304, 3072):
        x = torch.randn(M, P, device="cuda", dtype=dt)
        y = torch.randn(M, 32, device="cuda", dtype=dt)
        out = torch.zeros(P, 32, device="cuda", dtype=torch.float32)
        r = {"op": "lora_wgrad", "M": M, "P": P,
             "us": timed(lambda: K.lora_wgrad(x, y, out, 0.05, 7), (256, 512, 1024, 2048), "MIFT_WGRAD_BLOCKS")}
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
