#!/usr/bin/env python
"""Diagnostic: where do the eager and hipGraph-replayed training paths first differ?

Trains the same model/data with graph off / on (and graph on without the setup-time warm-up),
one optimizer step at a time, and prints per step the loss, the grad norm, the max |Δ| of the LoRA
grads (before the optimizer step zeroes them, via a pre-step hook) and of the parameters.

  python tools/diag_graph_eager.py [--model facebook/opt-125m] [--precision fp16] [--steps 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(model_name, precision, steps, graph, warm):
    import torch
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.parallel import dist as D
    from mift.train.trainer import TrainConfig, Trainer
    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16 if precision == "bf16" else torch.float16
    model = build_causal_lm(model_name, dtype=dtype, device=dev, seed=0)
    targets = ["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"] if "opt" in model_name else ["c_attn", "c_proj"]
    L.inject(model, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=targets))
    with torch.no_grad():
        for n, p in model.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.02, generator=torch.Generator(device=dev).manual_seed(len(n)))
    ds = synthetic_openwebtext(4 * 2 * steps, 128, model.config.vocab_size, model.config.pad_token_id, seed=3,
                               full_length=False)
    batcher = MicroBatcher(ds, 4, 2)
    ctx = D.init(verbose=False, sanity=False)
    tr = Trainer(model, batcher, TrainConfig(epochs=1, batch=4, accum=2, lr=1e-3, precision=precision,
                                             logging_steps=0, save_steps=0, step_log="none",
                                             graph="on" if graph else "off", warm_setup=warm), ctx)
    model.train()
    grads, params, losses, gns, infs = [], [], [], [], []
    real_step = tr.opt.step

    def hooked():
        grads.append(tr.arena.grad.detach().clone())
        real_step()
    tr.opt.step = hooked
    for mbs in batcher.epoch(0):
        loss, ntok = tr.train_step(mbs)
        st = tr.opt.stats()
        losses.append(float(loss) / ntok)
        gns.append(st["grad_norm"])
        infs.append(st["found_inf"])
        params.append(tr.arena.param.detach().clone())
    names = [(n, o, p.numel()) for (n, p), o in zip(tr.arena.named, tr.arena.offsets)]
    return {"loss": losses, "gn": gns, "inf": infs, "grads": grads, "params": params, "names": names}


def worst(a, b, names, k=4):
    """The k parameters whose slices differ most between two flat arena tensors."""
    d = (a - b).abs()
    per = sorted(((float(d[o:o + n].max()), nm) for nm, o, n in names), reverse=True)[:k]
    return [(nm, round(v, 6)) for v, nm in per if v > 0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="facebook/opt-125m")
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    runs = {"eager": run(a.model, a.precision, a.steps, False, True),
            "eager2": run(a.model, a.precision, a.steps, False, True),
            "graph": run(a.model, a.precision, a.steps, True, True),
            "graph_nowarm": run(a.model, a.precision, a.steps, True, False)}
    if a.precision == "fp16":
        os.environ["MIFT_DIAG_NOREBIND"] = "1"
        runs["graph_norebind"] = run(a.model, a.precision, a.steps, True, True)
    base = runs["eager"]
    for name, r in runs.items():
        rec = {"run": name, "loss": r["loss"], "gn": r["gn"], "found_inf": r["inf"]}
        rec["max_dgrad"] = [float((g - g0).abs().max()) for g, g0 in zip(r["grads"], base["grads"])]
        rec["max_dparam"] = [float((p - p0).abs().max()) for p, p0 in zip(r["params"], base["params"])]
        rec["worst_grad"] = [worst(g, g0, r["names"]) for g, g0 in zip(r["grads"], base["grads"])]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
