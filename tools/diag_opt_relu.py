#!/usr/bin/env python
"""Diagnostic for the OPT fused-vs-fp32 LoRA gradient gap: per-parameter relative errors with the
fc1 bias pushed to +-b (b = 0, 1, 2, 4) so the fc1 pre-activations move away from the ReLU kink.
Prints one JSON line per (dtype, b): the worst parameters and the fraction of fc1 pre-activations
within 16-bit rounding of zero.

  python tools/diag_opt_relu.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    import torch
    from mift import lora as L
    from test_fused_gpu import _opt_models
    for dtype in (torch.float16, torch.bfloat16):
        for b in (0.0, 1.0, 2.0, 4.0):
            cfg, ref, fused = _opt_models(dtype, 0.0, lora_p=0.0)
            with torch.no_grad():
                for m_ in (ref, fused):
                    for n, q in m_.named_parameters():
                        if n.endswith("fc1.bias") and b > 0:
                            sgn = torch.where(torch.arange(q.numel(), device=q.device) % 2 == 0, b, -b)
                            q.copy_(sgn.to(q.dtype))
            torch.manual_seed(1)
            ids = torch.randint(3, cfg.vocab_size, (3, 96), device="cuda")
            ref.train()
            fused.train()
            zs = []
            hooks = [m.fc1.register_forward_hook(lambda mod, i, o: zs.append(o.detach().float()))
                     for m in ref.model.decoder.layers]
            ref(input_ids=ids, labels=ids, reduction="sum")["loss"].backward()
            for h in hooks:
                h.remove()
            fused(input_ids=ids, labels=ids, reduction="sum")["loss"].backward()
            errs = []
            for (n1, p1), (_, p2) in zip(L.lora_parameters(ref), L.lora_parameters(fused)):
                g1, g2 = p1.grad.float(), p2.grad.float()
                errs.append((float((g1 - g2).norm() / (g1.norm() + 1e-6)), n1))
            errs.sort(reverse=True)
            tol = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
            near = [float((z.abs() < 4 * tol * z.abs().max()).float().mean()) for z in zs]
            print(json.dumps({"dtype": str(dtype), "fc1_bias": b, "worst": errs[:3], "near_kink_frac": near}),
                  flush=True)


if __name__ == "__main__":
    main()
