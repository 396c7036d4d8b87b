"""Tall-skinny LoRA projection [M,K] x [32,K]^T: lora_proj vs every gemm_nt tile vs torch.mm (hipBLASLt).

  python tools/bench_proj_gemm.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import mift  # noqa: E402
from mift.ops import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

C = mift._ext.require()
for (M, Kd) in [(24576, 2560), (24576, 7680), (24576, 10240), (8192, 2304), (8192, 768), (8192, 3072)]:
    x = torch.randn(M, Kd, device="cuda", dtype=torch.float16 if M > 8192 else torch.bfloat16)
    w = torch.zeros(32, Kd, device="cuda", dtype=x.dtype); w[:24] = 0.02 * torch.randn(24, Kd, device="cuda", dtype=x.dtype)
    r = {"M": M, "K": Kd}
    r["lora_proj"] = round(timeit(lambda: K.lora_proj(x, w, 1.0, 0.0, 0, rows=24)) * 1000, 1)
    for t in range(0, 16):
        try:
            out = C.gemm_nt(x, w, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, t, None, None, 0.0, 0)[0]
            ref = x.float() @ w.float().t()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            if err > 1e-2:
                r[f"t{t}"] = f"err{err:.2e}"; continue
            r[f"t{t}"] = round(timeit(lambda: C.gemm_nt(x, w, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, t, None, None, 0.0, 0)) * 1000, 1)
        except Exception as e:
            r[f"t{t}"] = "x"
    r["torch"] = round(timeit(lambda: torch.mm(x, w.t())) * 1000, 1)
    print(json.dumps(r), flush=True)
