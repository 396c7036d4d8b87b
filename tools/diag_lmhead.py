"""LM-head forward diagnostics: fused EPI 1 kernel with / without the E store (MIFT_LM_DBG) vs the
plain 256x256 GEMM and hipBLASLt at the distilgpt2 shape.  DIAG_QUICK=1: 2 launches each (PMC runs)."""
import os, sys, statistics, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mift._C as C
M, K, V = 8192, 768, 50257
Vp = 50304
a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(Vp, K, device="cuda", dtype=torch.bfloat16) * 0.02
lab = torch.randint(0, V, (M,), device="cuda")
def t(fn, iters=10 if not os.environ.get('DIAG_QUICK') else 2, rounds=5 if not os.environ.get('DIAG_QUICK') else 1):
    fn(); torch.cuda.synchronize(); ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters): fn()
        e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e) / iters * 1000)
    return statistics.median(ts)
R = 1 if os.environ.get('DIAG_QUICK') else 2
for r in range(R):
    row = {}
    for d in ("0", "1", "2", "3"):
        os.environ["MIFT_LM_DBG"] = d
        row["fused_dbg" + d] = round(t(lambda: C.lmhead_fwd(a, w, lab, V, 0, -1, None)), 1)
    for d in ("0", "1"):
        os.environ["MIFT_LM_DBG"] = d
        row["plain_t8_dbg" + d] = round(t(lambda: C.gemm_nt(a, w, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, 8, None, None, 0.0, 0)), 1)
    row["torch"] = round(t(lambda: torch.matmul(a, w.t())), 1)
    print(row, flush=True)

# tile raster A/B (MIFT_GEMM_GROUP, read per call) on the fused head and OPT-scale plain GEMMs
os.environ["MIFT_LM_DBG"] = "0"
shapes = [("lm_head", a, w)]
if not os.environ.get("DIAG_QUICK"):
    for nm, Mx, Nx, Kx in [("opt.fc1.fwd.mb48", 24576, 10240, 2560), ("opt.lm_head.mb8", 4096, 50304, 2560),
                           ("opt.qkv.fwd.mb48", 24576, 7680, 2560)]:
        shapes.append((nm, torch.randn(Mx, Kx, device="cuda", dtype=torch.float16),
                       torch.randn(Nx, Kx, device="cuda", dtype=torch.float16) * 0.02))
for nm, x, wt in shapes:
    res = {}
    for g in ("0", "2", "4", "8"):
        os.environ["MIFT_GEMM_GROUP"] = g
        if nm == "lm_head":
            res["fused_g" + g] = round(t(lambda: C.lmhead_fwd(x, wt, lab, V, 0, -1, None)), 1)
        res["plain_g" + g] = round(t(lambda: C.gemm_nt(x, wt, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0)), 1)
    os.environ.pop("MIFT_GEMM_GROUP")
    res["torch"] = round(t(lambda: torch.matmul(x, wt.t())), 1)
    print(nm, res, flush=True)
