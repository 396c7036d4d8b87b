"""LM-head dgrad (EPI 2) with and without its per-column-group accumulator rescale (MIFT_LM_DBG bit 3:
timing only, wrong numbers) and over the split-K count (MIFT_LM_SPLIT), distilgpt2 and OPT-2.7B shapes,
interleaved rounds in one process."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mift.ops import kernels as K  # noqa: E402


def timeit(fn, iters=10, rounds=3):
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
        ts.append(s.elapsed_time(e) / iters)
    return statistics.median(ts)


def main():
    for M, d, V, dt in ((8192, 768, 50257, torch.bfloat16), (6144, 2560, 50272, torch.float16)):
        Vp = (V + 63) // 64 * 64
        a = torch.randn(M, d, device="cuda", dtype=dt)
        w = (torch.randn(Vp, d, device="cuda", dtype=dt) * 0.05)
        wt = w.t().contiguous()
        lab = torch.randint(0, V, (M,), device="cuda")
        E, stats, lse, loss, zlab = K.lmhead_fwd(a, w, lab, V)[:5]
        g = torch.ones(1, device="cuda")
        res = {}
        arms = {"default": {}, "no_rescale": {"MIFT_LM_DBG": "8"}}
        for sp in (4, 6, 7, 8, 10, 12):
            arms[f"split{sp}"] = {"MIFT_LM_SPLIT": str(sp)}
        for _ in range(3):
            for name, env in arms.items():
                os.environ.update(env)
                res.setdefault(name, []).append(timeit(lambda: K.lmhead_dgrad(E, wt, w, lab, V, stats, lse, g)))
                for k in env:
                    os.environ.pop(k, None)
        print(json.dumps({"M": M, "d": d, "V": V, **{k + "_us": round(min(v) * 1e3, 1) for k, v in res.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
