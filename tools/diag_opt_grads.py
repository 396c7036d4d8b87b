"""Print per-parameter LoRA grad errors of the fused OPT path vs the fp32 reference."""
import sys
sys.path[:0] = [".", "tests"]
import torch
from test_fused_gpu import _opt_models
from mift import lora as L

for dt in (torch.float16, torch.bfloat16):
    for p in (0.0, 0.1):
        cfg, ref, fused = _opt_models(dt, p, 0.05 if p else 0.0)
        torch.manual_seed(1)
        ids = torch.randint(3, cfg.vocab_size, (3, 96), device="cuda")
        ref.train(); fused.train()
        lr = ref(input_ids=ids, labels=ids, reduction="sum")["loss"]; lr.backward()
        lf = fused(input_ids=ids, labels=ids, reduction="sum")["loss"]; lf.backward()
        print(dt, p, "loss", lr.item(), lf.item())
        for (n1, p1), (n2, p2) in zip(L.lora_parameters(ref), L.lora_parameters(fused)):
            g1, g2 = p1.grad.float(), p2.grad.float()
            print(f"  {n1[14:]:45s} |g|={g1.norm():.3e} rel={((g1-g2).norm()/(g1.norm()+1e-12)):.3e}")
