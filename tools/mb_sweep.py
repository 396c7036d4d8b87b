#!/usr/bin/env python
"""dp1 tokens/s of a LoRA fine-tune step as a function of the micro-batch size.

One process, one GPU, no pipeline: for every micro-batch size mb the same 96 x 512-token optimizer
step (P2's batch 1 x accum 96) is regrouped into 96/mb micro-batches and timed on a fresh model +
Trainer (graph-replayed steps).  The per-micro-batch cost curve is the input of the pipeline
micro-batch planner (mift.parallel.plan): a stage of a PP run executes exactly these micro-batches.

  python tools/mb_sweep.py --model facebook/opt-2.7b --mbs 1,2,4,8,12,16,24,48 --steps 3 --warmup 2

Prints one JSON line per micro-batch size: {"model", "mb", "ms_per_step", "ms_per_seq", "tok_s", "max_mem_gib"}.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_one(model_name, mb, seq, per_step, steps, warmup, precision):
    import torch
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.parallel import dist as D
    from mift.train.trainer import TrainConfig, Trainer

    ctx = D.init(verbose=False, sanity=False)
    dtype = torch.float16 if precision == "fp16" else torch.bfloat16
    is_opt = "opt" in model_name.lower()
    m = build_causal_lm(model_name, dtype=dtype, device=ctx.device, seed=0)
    targets = ["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"] if is_opt else ["c_attn", "c_proj"]
    L.inject(m, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=targets))
    acc = per_step // mb
    ds = synthetic_openwebtext(per_step * (steps + warmup), seq, m.config.vocab_size, m.config.pad_token_id,
                               seed=1234, full_length=True)
    batcher = MicroBatcher(ds, mb, acc)
    torch.cuda.reset_peak_memory_stats()
    tr = Trainer(m, batcher, TrainConfig(epochs=1, batch=mb, accum=acc, lr=5e-5, precision=precision,
                                         logging_steps=0, save_steps=0, step_log="none"), ctx)
    m.train()
    st = list(batcher.epoch(0))
    for i in range(warmup):
        tr.train_step(st[i])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        tr.train_step(st[i])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    mem = torch.cuda.max_memory_allocated() / 2 ** 30
    if tr.reducer is not None:
        tr.reducer.remove()
    del tr, m, st, batcher, ds
    torch.cuda.empty_cache()
    return {"model": model_name, "mb": mb, "seq": seq, "per_step": per_step, "ms_per_step": round(dt * 1e3, 2),
            "ms_per_seq": round(dt * 1e3 / per_step, 4), "tok_s": round(per_step * seq / dt, 1),
            "max_mem_gib": round(mem, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="facebook/opt-2.7b")
    ap.add_argument("--mbs", default="1,2,4,8,12,16,24,48")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--per_step", type=int, default=96)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    for mb in [int(x) for x in a.mbs.split(",")]:
        r = run_one(a.model, mb, a.seq, a.per_step, a.steps, a.warmup, a.precision)
        line = json.dumps(r)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")


if __name__ == "__main__":
    main()
