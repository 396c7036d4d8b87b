"""Which hipBLASLt kernels torch.matmul runs for the OPT-2.7B layer GEMMs (fp16, M = 6144 / 24576): run
under rocprofv3 --kernel-trace; the Tensile kernel names encode macro tile, depth, wave layout and
prefetch settings (reference point for the phased 256x256 kernel, which trails them by 8-19 %)."""
import torch

from bench_kernels import OPT_LAYER

for M in (6144, 24576):
    for name, N, K in OPT_LAYER:
        a = torch.randn(M, K, device="cuda", dtype=torch.float16)
        b = torch.randn(N, K, device="cuda", dtype=torch.float16)
        for _ in range(3):
            torch.matmul(a, b.t())
        torch.cuda.synchronize()
        print(name, M, N, K, flush=True)
