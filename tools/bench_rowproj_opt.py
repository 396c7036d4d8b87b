"""The fused LoRA row passes at the OPT widths (rowproj.hip MFMA form on 8 / 16 waves) against the
separate passes they replace in an OPT training step (fp16, micro-batch 12 x 512 = 6144 rows):

  fwd  LN + q/k/v (or fc1) input projection:  layer_norm_fwd_proj   vs  layer_norm_fwd + lora_proj
  bwd  LN-bwd + residual-dropout-bwd + dT:     ln_bwd_mask_proj      vs  layer_norm_bwd + mask_scale + lora_proj
  bwd  residual-dropout-bwd + dT:              mask_proj             vs  mask_scale + lora_proj
  plain projection (out_proj input):           lora_proj (MODE 2)    vs  lora_proj's own kernel (MIFT_ROWPROJ_V=1)

  python tools/bench_rowproj_opt.py [--json out.json]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--M", type=int, default=6144)
    a = ap.parse_args()
    mift._ext.require()
    dev, dt, M = "cuda", torch.float16, a.M
    rows = []
    for D, rank in ((2560, 24), (2560, 8), (4096, 24), (2048, 24)):
        torch.manual_seed(0)
        x = torch.randn(M, D, device=dev).to(dt)
        dy = torch.randn(M, D, device=dev).to(dt)
        dres = torch.randn(M, D, device=dev).to(dt)
        lw = (1 + 0.1 * torch.randn(D, device=dev)).to(dt)
        lb = (0.1 * torch.randn(D, device=dev)).to(dt)
        pw = torch.zeros(32, D, device=dev, dtype=dt)
        pw[:rank] = (torch.randn(rank, D, device=dev) * 0.02).to(dt)
        _, mean, rstd = K.layer_norm_fwd(x, lw, lb, 1e-5)
        r = {"M": M, "D": D, "rows": rank}

        def t(fn):
            return round(timeit(fn) * 1e3, 1)

        r["ln_fwd_proj_us"] = t(lambda: K.layer_norm_fwd_proj(x, lw, lb, 1e-5, pw, rank, 1.0, 0.05, 7))
        r["ln_fwd+lora_proj_us"] = t(lambda: (K.layer_norm_fwd(x, lw, lb, 1e-5),
                                              K.lora_proj(x, pw, 1.0, 0.05, 7, rows=rank)))
        if D != 4096:  # the LN-bwd row pass spills at 4096 and is not built there (rowproj.hip)
            r["ln_bwd_mask_proj_us"] = t(lambda: K.ln_bwd_mask_proj(dy, x, lw, mean, rstd, dres, 0.1, 7, pw, rank, 1.0))
        r["ln_bwd+mask_scale+lora_proj_us"] = t(lambda: (K.layer_norm_bwd(dy, x, lw, mean, rstd, dres=dres),
                                                         K.mask_scale(dy, 0.1, 7),
                                                         K.lora_proj(dy, pw, 1.0, 0.0, 0, rows=rank)))
        r["mask_proj_us"] = t(lambda: K.mask_proj(dy, 0.1, 7, pw, rank, 1.0))
        r["mask_scale+lora_proj_us"] = t(lambda: (K.mask_scale(dy, 0.1, 7), K.lora_proj(dy, pw, 1.0, 0.0, 0, rows=rank)))
        r["lora_proj_mfma_us"] = t(lambda: K.lora_proj(x, pw, 1.0, 0.05, 7, rows=rank))
        os.environ["MIFT_ROWPROJ_V"] = "1"
        r["lora_proj_own_us"] = t(lambda: K.lora_proj(x, pw, 1.0, 0.05, 7, rows=rank))
        r["ln_fwd_proj_rowkernel_us"] = t(lambda: K.layer_norm_fwd_proj(x, lw, lb, 1e-5, pw, rank, 1.0, 0.05, 7))
        os.environ.pop("MIFT_ROWPROJ_V")
        r["hbm_floor_ln_bwd_mask_proj_us"] = round(5 * M * D * 2 / 6.0e12 * 1e6, 1)  # dy, x, dres in; dh, y out
        print(json.dumps(r), flush=True)
        rows.append(r)
    # the fused q/k/v dgrad's dT projection: plain MODE 2 over the 3*2560-wide gradient
    for m in (M, 4 * M):
        torch.manual_seed(0)
        g = torch.randn(m, 7680, device=dev).to(dt)
        pw = torch.zeros(32, 7680, device=dev, dtype=dt)
        pw[:24] = (torch.randn(24, 7680, device=dev) * 0.02).to(dt)
        r = {"M": m, "D": 7680, "rows": 24}
        r["lora_proj_mfma_us"] = round(timeit(lambda: K.lora_proj(g, pw, 1.0, 0.0, 0, rows=24)) * 1e3, 1)
        os.environ["MIFT_ROWPROJ_V"] = "1"
        r["lora_proj_own_us"] = round(timeit(lambda: K.lora_proj(g, pw, 1.0, 0.0, 0, rows=24)) * 1e3, 1)
        os.environ.pop("MIFT_ROWPROJ_V")
        r["hbm_floor_us"] = round(m * 7680 * 2 / 6.0e12 * 1e6, 1)
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
