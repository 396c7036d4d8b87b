"""Fused LM-head forward (lmhead_fwd: GEMM + exp epilogue + E store + lse) alone at the distilgpt2
and OPT-2.7B mb8 shapes: median of 5 rounds x 10 launches, random data."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mift.ops import kernels as K  # noqa: E402

for name, M, d, V, dt in [("distilgpt2", 8192, 768, 50257, torch.bfloat16), ("opt-2.7b.mb8", 4096, 2560, 50272, torch.float16)]:
    Vp = (V + 63) // 64 * 64
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, d, device="cuda", generator=g).to(dt)
    W = torch.zeros(Vp, d, device="cuda", dtype=dt)
    W[:V] = (0.05 * torch.randn(V, d, device="cuda", generator=g)).to(dt)
    lab = torch.randint(0, V, (M,), device="cuda", generator=g)
    outs, ts = {}, {"full": [], "generic": []}
    for arm, dbg in (("full", "0"), ("generic", "4")):
        os.environ["MIFT_LM_DBG"] = dbg
        outs[arm] = K.lmhead_fwd(x, W, lab, V)
    for _ in range(5):
        for arm, dbg in (("full", "0"), ("generic", "4")):  # interleaved arms (same process)
            os.environ["MIFT_LM_DBG"] = dbg
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                K.lmhead_fwd(x, W, lab, V)
            b.record()
            torch.cuda.synchronize()
            ts[arm].append(a.elapsed_time(b) * 100)
    os.environ.pop("MIFT_LM_DBG", None)
    same = all(torch.equal(p, q) for p, q in zip(outs["full"], outs["generic"]))
    print(json.dumps({"name": name, "full_us": round(statistics.median(ts["full"]), 1),
                      "generic_us": round(statistics.median(ts["generic"]), 1), "bit_identical": same}), flush=True)
