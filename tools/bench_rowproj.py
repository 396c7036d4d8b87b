"""Row-projection kernels at the OPT-2.7B / distilgpt2 training shapes.

Compares, per shape, the LoRA input projection variants:
  ln_fwd_proj(LR)        LN + projection in one row pass (csrc/kernels/rowproj.hip)
  ln_fwd + lora_proj     LN, then the MFMA tall-skinny projection (csrc/kernels/lora.hip)
  lora_proj / mask_proj  stand-alone projections (forward T, backward dT)
  torch.mm               hipBLASLt x @ W^T for the same [M,32] product (reference point)
and reports us and effective HBM GB/s (bytes of x read once + outputs written).

  python tools/bench_rowproj.py [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import mift  # noqa: E402
from mift.ops import kernels as K  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

SHAPES = [  # (name, M, D, rank rows, dtype)
    ("opt.qkv.ln_proj", 24576, 2560, 24, torch.float16),
    ("opt.fc1.ln_proj", 24576, 2560, 8, torch.float16),
    ("opt.out.proj", 24576, 2560, 8, torch.float16),
    ("opt.fc2.proj", 24576, 10240, 8, torch.float16),
    ("opt.qkv.dT", 24576, 7680, 24, torch.float16),
    ("dgpt.c_attn.ln_proj", 8192, 768, 8, torch.bfloat16),
    ("dgpt.c_fc.dT", 8192, 3072, 8, torch.bfloat16),
    ("opt125.qkv.ln_proj", 16384, 768, 28, torch.float16),
    ("dgpt.c_attn.dT", 8192, 2304, 8, torch.bfloat16),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    assert mift.kernels_available(), mift._ext.error()
    dev = torch.device("cuda", 0)
    res = []
    for name, M, D, r, dt in SHAPES:
        x = torch.randn(M, D, device=dev, dtype=dt)
        lw = torch.rand(D, device=dev, dtype=dt) + 0.5
        lb = torch.randn(D, device=dev, dtype=dt) * 0.1
        w32 = torch.zeros(32, D, device=dev, dtype=dt)
        w32[:r] = torch.randn(r, D, device=dev, dtype=dt) * 0.02
        gb = (M * D * x.element_size()) / 1e9
        row = {"name": name, "M": M, "D": D, "rows": r}
        if D <= 4096:  # the one-wave-per-row producers hold a whole row in registers
            t = timeit(lambda: K.layer_norm_fwd_proj(x, lw, lb, 1e-5, w32, r, 1.0, 0.05, 7))
            row["ln_fwd_proj_us"] = round(t * 1e3, 1)
            t = timeit(lambda: K.layer_norm_fwd(x, lw, lb, 1e-5))
            row["ln_fwd_us"] = round(t * 1e3, 1)
            t = timeit(lambda: K.mask_proj(x, 0.1, 7, w32, r, 1.0))
            row["mask_proj_us"] = round(t * 1e3, 1)
            t = timeit(lambda: K.mask_scale(x, 0.1, 7))
            row["mask_scale_us"] = round(t * 1e3, 1)
            if D in (768, 1024):  # the MFMA 16-row form runs by default there; the row kernels for A/B
                os.environ["MIFT_ROWPROJ_V"] = "1"
                t = timeit(lambda: K.layer_norm_fwd_proj(x, lw, lb, 1e-5, w32, r, 1.0, 0.05, 7))
                row["ln_fwd_proj_rowkernel_us"] = round(t * 1e3, 1)
                t = timeit(lambda: K.mask_proj(x, 0.1, 7, w32, r, 1.0))
                row["mask_proj_rowkernel_us"] = round(t * 1e3, 1)
                os.environ.pop("MIFT_ROWPROJ_V")
        t = timeit(lambda: K.lora_proj(x, w32, 1.0, 0.05, 7))
        row["lora_proj_p_us"] = round(t * 1e3, 1)
        t = timeit(lambda: K.lora_proj(x, w32, 1.0, 0.0, 0))
        row["lora_proj_us"] = round(t * 1e3, 1)
        if D in (768, 1024, 2304):  # rowproj MFMA form by default; lora_proj's own kernel for A/B
            os.environ["MIFT_ROWPROJ_V"] = "1"
            t1 = timeit(lambda: K.lora_proj(x, w32, 1.0, 0.05, 7))
            row["lora_proj_p_oldkernel_us"] = round(t1 * 1e3, 1)
            os.environ.pop("MIFT_ROWPROJ_V")
        row["lora_proj_GBps"] = round(gb / (t * 1e-3), 0)
        t = timeit(lambda: torch.mm(x, w32.t()))
        row["torch_mm_us"] = round(t * 1e3, 1)
        # numerics of the projection (p = 0) vs fp32 torch
        ref = x.float() @ w32.float().t()
        got = K.lora_proj(x, w32, 1.0, 0.0, 0).float()
        row["lora_proj_maxerr"] = float((got - ref).abs().max())
        print(json.dumps(row), flush=True)
        res.append(row)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
