#!/usr/bin/env python
"""Diagnostic: where do two eager DP replicas (fused GPU path, gloo) first disagree?

Each rank checksums its all-reduced LoRA grads right before every optimizer step (and its params
right after), the per-rank values are gathered on rank 0 and the first differing arena slices are
named together with the reducer's bucket launch log of that step.

  python tools/diag_ddp_eager.py [--graph 0] [--steps 3] [--max_grad_norm 1e-3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, world, graph=False, steps=3, max_grad_norm=1e-3, bucket_mb=25.0):
    import torch
    import torch.distributed as dist
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.models.opt import OPTConfig
    from mift.parallel import dist as D
    from mift.train.trainer import TrainConfig, Trainer
    ctx = D.init(verbose=False, sanity=True)
    cfg = OPTConfig.preset("opt-tiny")
    model = build_causal_lm("opt-tiny", dtype=torch.float16, device=ctx.device, seed=3)
    model.config.dropout = 0.1
    L.inject(model, L.LoraConfig(r=4, lora_alpha=8, lora_dropout=0.05,
                                 target_modules=["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"]), seed=3)
    model.seed = 11
    mb, accum = 2, 6
    ds = synthetic_openwebtext(mb * accum * steps * ctx.dp, 64, cfg.vocab_size, cfg.pad_token_id, seed=5,
                               full_length=False, mean_tokens=40)
    batcher = MicroBatcher(ds, mb, accum, rank=ctx.dp_rank, world=ctx.dp)
    tc = TrainConfig(epochs=1, batch=mb, accum=accum, lr=1e-3, max_steps=steps, precision="fp16", logging_steps=1,
                     step_log="none", save_steps=0, graph="on" if graph else "off", max_grad_norm=max_grad_norm)
    tr = Trainer(model, batcher, tc, ctx)
    names = [(n, o, p.numel()) for (n, p), o in zip(tr.arena.named, tr.arena.offsets)]
    off2name = {o: n for n, o, _ in names}
    events = []  # notification / launch order of the current step (last micro-step only counts)
    red = tr.reducer
    r_ready, r_launch = red._on_ready_offsets, red._launch

    def on_ready(offsets):
        events.append(("fused", [off2name.get(o, o) for o in offsets], red._sync))
        r_ready(offsets)


    def launch(b, where="finish"):
        events.append(("LAUNCH", b["idx"], where))
        r_launch(b, where)
    red._on_ready_offsets = on_ready
    tr.arena.grad_ready = on_ready
    for n, p in tr.arena.named:  # the reducer's own hooks were bound at construction: log beside them
        p.register_post_accumulate_grad_hook(lambda _p, n=n: events.append(("hook", n, red._sync)))
    red._launch = launch
    recs = []
    real_step = tr.opt.step

    def hooked():
        (torch.cuda.synchronize() if torch.cuda.is_available() else None)
        recs.append({"grad": tr.arena.grad.detach().cpu().clone(),
                     "log": [e for e in events if e[0] == "LAUNCH" or e[2]]})
        events.clear()
        real_step()
        (torch.cuda.synchronize() if torch.cuda.is_available() else None)
        recs[-1]["param"] = tr.arena.param.detach().cpu().clone()
    tr.opt.step = hooked
    model.train()
    for mbs in batcher.epoch(0):
        tr.train_step(mbs)
        if tr.global_step >= steps:
            break
    out = [None] * world
    dist.all_gather_object(out, recs)
    D.destroy()
    if rank != 0:
        return None
    rep = []
    for s in range(len(recs)):
        a, b = out[0][s], out[1][s]
        r = {"step": s + 1, "log0": a["log"], "log1": b["log"]}
        for key in ("grad", "param"):
            d = (a[key] - b[key]).abs()
            bad = [(nm, float(d[o:o + n].max())) for nm, o, n in names if float(d[o:o + n].max()) > 0]
            r[key + "_diff_tensors"] = len(bad)
            r[key + "_first"] = bad[:4]
        rep.append(r)
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--max_grad_norm", type=float, default=1e-3)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    from mift.utils import harness
    env = {"MIFT_DEVICE": a.device, "MIFT_BACKEND": "gloo"}
    res = harness.run(_worker, 2, env=env, timeout=240, graph=bool(a.graph), steps=a.steps,
                      max_grad_norm=a.max_grad_norm)
    for r in res[0]:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
