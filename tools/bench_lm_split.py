"""LM-head dgrad split-K count (MIFT_LM_SPLIT) sweep at the distilgpt2 shape: dgrad kernel + slab
reduction time per S, interleaved rounds in one process."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mift.ops import kernels as K  # noqa: E402

M, d, V = 8192, 768, 50257
Vp = (V + 63) // 64 * 64
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(M, d, device="cuda", generator=g).to(torch.bfloat16)
W = torch.zeros(Vp, d, device="cuda", dtype=torch.bfloat16)
W[:V] = (0.05 * torch.randn(V, d, device="cuda", generator=g)).to(torch.bfloat16)
Wt = W.t().contiguous()
lab = torch.randint(0, V, (M,), device="cuda", generator=g)
gs = torch.full((1,), 1.0 / M, device="cuda")
E, st, lse, loss, zl = K.lmhead_fwd(x, W, lab, V)
ref = None
res = {}
for rnd in range(4):
    for S in (3, 4, 5, 6, 8, 10):
        os.environ["MIFT_LM_SPLIT"] = str(S)
        out = K.lmhead_dgrad(E, Wt, W, lab, V, st, lse, gs)
        if ref is None:
            ref = out.float()
        err = float((out.float() - ref).norm() / ref.norm())
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            K.lmhead_dgrad(E, Wt, W, lab, V, st, lse, gs)
        b.record()
        torch.cuda.synchronize()
        res.setdefault(S, []).append(a.elapsed_time(b) * 100)
        res.setdefault(f"err{S}", []).append(err)
os.environ.pop("MIFT_LM_SPLIT", None)
print(json.dumps({str(k): round(statistics.median(v), 6 if str(k).startswith("err") else 1) for k, v in res.items()}))
