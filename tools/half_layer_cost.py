"""Cost of an OPT decoder layer's attention and MLP sub-blocks (the half-layer pipeline units,
parallel/pipeline.py ``partition_layers(..., "halves")``): forward + backward of a stage holding
layers [0, 0.5) (attention), [0.5, 1) (MLP), [0, 1) and [0, 2) on the fused path, LoRA on all six
linears, at the BASELINE configs' micro-batches.  Prints the attention share to use as
MIFT_PP_ATTN_FRAC / pipeline.ATTN_FRACTION.

  python tools/half_layer_cost.py [--model opt-2.7b --mb 12]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="opt-2.7b")
    ap.add_argument("--mb", type=int, default=12)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import torch
    from mift import lora as L
    from mift.models import build_causal_lm
    torch.manual_seed(0)
    dev = torch.device("cuda")
    res = {}
    ranges = {"attn": (0, 0.5), "mlp": (0.5, 1), "layer": (0, 1), "two_layers": (0, 2)}
    models = {}
    for name, rg in ranges.items():
        m = build_causal_lm(a.model, dtype=torch.float16, device=dev, seed=0, layer_range=rg, has_embed=False,
                            has_head=False)
        L.inject(m, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05,
                                 target_modules=["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"]))
        m.train()
        models[name] = m
    d = models["layer"].config.hidden_size
    h0 = torch.randn(a.mb, a.seq, d, device=dev, dtype=torch.float16)
    mask = torch.ones(a.mb, a.seq, device=dev, dtype=torch.long)
    g = torch.randn_like(h0) * 1e-2

    def step(m):
        h = h0.detach().requires_grad_(True)
        out = m(attention_mask=mask, hidden_states=h)["hidden_states"]
        out.backward(g)

    for _ in range(2):
        for m in models.values():
            step(m)
    torch.cuda.synchronize()
    for _ in range(5):
        for name, m in models.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                step(m)
            e.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(s.elapsed_time(e) / a.iters)
    med = {k: round(statistics.median(v), 3) for k, v in res.items()}
    out = {"model": a.model, "micro_batch": a.mb, "seq": a.seq, "ms_fwd_bwd": med,
           "attn_fraction": round(med["attn"] / (med["attn"] + med["mlp"]), 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
