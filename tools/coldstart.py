#!/usr/bin/env python
"""Cold-start breakdown of the distilgpt2 LoRA training run in a FRESH process.

Prints one JSON line with host wall-clock (synchronised) for: import, process-group init, model
build + LoRA inject, Trainer construction (includes the setup-time warm-up / graph capture when
enabled), and each of the first --steps optimizer steps, then the steady-state mean.

  python tools/coldstart.py [--steps 12] [--warm_setup 0|1]
"""
import argparse
import json
import os
import sys
import time

T0 = time.perf_counter()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warm_setup", type=int, default=None, help="override TrainConfig.warm_setup")
    ap.add_argument("--model", default="distilgpt2")
    a = ap.parse_args()
    rec = {}
    t = time.perf_counter()
    import torch
    import mift
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.parallel import dist as D
    from mift.train.trainer import TrainConfig, Trainer
    rec["import_s"] = time.perf_counter() - t
    t = time.perf_counter()
    ctx = D.init(verbose=False, sanity=True)
    torch.cuda.synchronize()
    rec["init_s"] = time.perf_counter() - t
    t = time.perf_counter()
    model = build_causal_lm(a.model, dtype=torch.bfloat16, device=ctx.device, seed=0)
    L.inject(model, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=["c_attn", "c_proj"]))
    torch.cuda.synchronize()
    rec["model_s"] = time.perf_counter() - t
    ds = synthetic_openwebtext(32 * (a.steps + 2), 256, model.config.vocab_size, model.config.pad_token_id,
                               seed=1234, full_length=True)
    batcher = MicroBatcher(ds, 32, 1, rank=0, world=1)
    kw = {} if a.warm_setup is None else {"warm_setup": bool(a.warm_setup)}
    t = time.perf_counter()
    tr = Trainer(model, batcher, TrainConfig(epochs=1, batch=32, accum=1, lr=5e-5, logging_steps=0, save_steps=0,
                                             step_log="none", **kw), ctx)
    torch.cuda.synchronize()
    rec["trainer_setup_s"] = time.perf_counter() - t
    model.train()
    steps = list(batcher.epoch(0))
    per = []
    for i in range(min(a.steps, len(steps))):
        t = time.perf_counter()
        tr.train_step(steps[i])
        torch.cuda.synchronize()
        per.append(round((time.perf_counter() - t) * 1000, 3))
    rec["step_ms"] = per
    tail = per[len(per) // 2:]
    rec["steady_ms"] = round(sum(tail) / max(1, len(tail)), 3)
    rec["first_step_excess_ms"] = round(sum(per) - rec["steady_ms"] * len(per), 1)
    rec["process_to_first_step_s"] = round(time.perf_counter() - T0, 3)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in rec.items()}), flush=True)
    D.destroy()


if __name__ == "__main__":
    main()
