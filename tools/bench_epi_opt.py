import os, sys, json
sys.path.insert(0, "/root/repo")
import torch, mift
from tools.bench_kernels import timeit
C = mift._ext.require()
M, N, K = 24576, 10240, 2560
dt = torch.float16
a = torch.randn(M, K, device="cuda", dtype=dt); b = torch.randn(N, K, device="cuda", dtype=dt) / K ** 0.5
bias = torch.randn(N, device="cuda", dtype=dt); a2 = torch.randn(M, 32, device="cuda", dtype=dt); b2 = torch.randn(N, 32, device="cuda", dtype=dt)
aux = torch.randn(M, N, device="cuda", dtype=dt)
V = {
 "plain": lambda: C.gemm_nt(a, b, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0),
 "bias": lambda: C.gemm_nt(a, b, bias, None, None, 0, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0),
 "bias+relu": lambda: C.gemm_nt(a, b, bias, None, None, 2, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0),
 "ext": lambda: C.gemm_nt(a, b, None, a2, b2, 0, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0),
 "ext+bias+relu": lambda: C.gemm_nt(a, b, bias, a2, b2, 2, None, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0),
 "relubwd(aux)": lambda: C.gemm_nt(a, b, None, None, None, 5, aux, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.0, 0),
 "maskext+relubwd": lambda: C.gemm_nt(a, b, None, a2, b2, 5, aux, None, 0.0, 0, False, 1.0, None, 0, None, None, 0.05, 7),
 "torch": lambda: torch.matmul(a, b.t()),
}
res = {k: [] for k in V}
for _ in range(3):
    for k, f in V.items():
        res[k].append(timeit(f, rounds=3))
fl = 2.0 * M * N * K
for k, v in res.items():
    t = min(v)
    print(f"{k:20s} {t*1e3:8.1f} us {fl/t/1e9:7.1f} TF/s", flush=True)
