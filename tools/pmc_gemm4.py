"""PMC target: tile 8 and tile 10 on one OPT shape (fp16, M 6144, N 7680, K 2560), 5 launches each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mift  # noqa: E402
import mift._C as C  # noqa: E402

a = torch.randn(6144, 2560, device="cuda", dtype=torch.float16)
b = torch.randn(7680, 2560, device="cuda", dtype=torch.float16)
for tile in (8, 10):
    for _ in range(5):
        C.gemm_nt(a, b, None, None, None, 0, None, None, 0.0, 0, False, 1.0, None, tile, None, None, 0.0, 0)
torch.cuda.synchronize()
print("ok")
