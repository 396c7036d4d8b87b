#!/usr/bin/env python
"""Rehearse the BASELINE pipeline configs at REAL model size on one MI355X (VERDICT r2 #4c).

Every rank of the pipeline (and DP) grid is its own process on the same GPU; the transport is
gloo (host-staged) instead of RCCL, but the engine, its 1F1B schedule, the per-link p2p layout,
the ring buffers, the per-slot stage hipGraphs, the cross-stage grad-norm all-reduce and the
DP all-reduce run exactly the production code path.  The same data / seeds are first trained
by the same DP degree without pipelining (dp1 for PP4 / PP8, dp2 for 2dp×4pp); the PP run's loss
and grad-norm trajectories must match it.

  python tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 [--dp 1] --seq 512 --mb 4 --accum 24 --steps 3

Prints one JSON line (both trajectories, their max relative differences, per-step wall times).
Reference: Cluster/Project 2 - Course Project/finetune_lora_opt_pp.py:114-224.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, world, model="facebook/opt-2.7b", pp=1, seq=512, mb=4, accum=24, steps=3, graph="auto",
            partition="uniform", virtual=1):
    import torch
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.models.opt import OPTConfig
    from mift.parallel import dist as D
    from mift.parallel.pipeline import attn_cost_fraction, head_cost_layers, partition_layers, stage_chunks
    from mift.train.trainer import TrainConfig, Trainer

    ctx = D.init(pp=pp, verbose=False, sanity=True, virtual=virtual)
    cfg = OPTConfig.preset(model)
    kw = {}
    split = None
    if ctx.pp > 1:
        V = ctx.pp_virtual
        split = partition_layers(cfg.num_hidden_layers, ctx.pp * V, partition, head_cost_layers(cfg), ranks=ctx.pp,
                                 attn_frac=attn_cost_fraction(cfg))
        ch = stage_chunks(split, ctx.pp, V, ctx.pp_rank)
        kw = dict(layer_range=ch if V > 1 else ch[0], has_embed=ctx.is_first_stage, has_head=ctx.is_last_stage)
    m = build_causal_lm(model, dtype=torch.float16, device=ctx.device, seed=0, **kw)
    L.inject(m, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05,
                             target_modules=["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"]))
    # global batch = mb * accum sequences per optimizer step, split over the DP replicas
    acc_r = accum // ctx.dp
    ds = synthetic_openwebtext(mb * accum * steps, seq, cfg.vocab_size, cfg.pad_token_id, seed=1234,
                               full_length=True)
    batcher = MicroBatcher(ds, mb, acc_r, rank=ctx.dp_rank, world=ctx.dp)
    tr = Trainer(m, batcher, TrainConfig(epochs=1, batch=mb, accum=acc_r, lr=5e-5, precision="fp16",
                                         logging_steps=1, step_log="none", save_steps=0, max_steps=steps,
                                         graph=graph), ctx)
    m.train()
    losses, gns, times = [], [], []
    for mbs in batcher.epoch(0):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss, ntok = tr.train_step(mbs)
        torch.cuda.synchronize()
        times.append(round(time.perf_counter() - t0, 3))
        losses.append(tr._loss_for_log(loss) / max(1, ntok))
        gns.append(float(tr.opt.stats()["grad_norm"]))
        if tr.global_step >= steps:
            break
    stats = dict(tr.engine.stats) if tr.engine is not None else {}
    mem = torch.cuda.max_memory_allocated() / 2 ** 30
    D.destroy()
    return {"loss": losses, "grad_norm": gns, "step_s": times, "split": split, "engine": stats,
            "max_mem_gib": round(mem, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="facebook/opt-2.7b")
    ap.add_argument("--pp", type=int, default=4)
    ap.add_argument("--dp", type=int, default=1)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--mb", type=int, default=4)
    ap.add_argument("--accum", type=int, default=24)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--partition", default="uniform")
    ap.add_argument("--virtual", type=int, default=1, help="interleaved 1F1B model chunks per pipeline rank")
    ap.add_argument("--skip_ref", action="store_true")
    ap.add_argument("--timeout", type=int, default=900)
    a = ap.parse_args()
    from mift.utils import harness
    env = {"MIFT_DEVICE": "cuda", "MIFT_BACKEND": "gloo", "OMP_NUM_THREADS": "2"}
    kw = dict(model=a.model, seq=a.seq, mb=a.mb, accum=a.accum, steps=a.steps, partition=a.partition)
    out = {"model": a.model, "grid": f"dp{a.dp}xpp{a.pp}" + (f"xv{a.virtual}" if a.virtual > 1 else ""), "seq": a.seq, "micro_batch": f"{a.mb}x{a.accum}",
           "transport": "gloo (one GPU, every rank its own process)"}
    t = time.perf_counter()
    if not a.skip_ref:
        # reference: the same DP degree without pipelining (dp1 for a pure PP grid).  A dp2 grid
        # shards the data by replica, so its steps see other lines than a dp1 run's steps would.
        ref = harness.run(_worker, a.dp, env=env, timeout=a.timeout, pp=1, **kw)[0]
        out[f"dp{a.dp}"] = ref
        print(f"dp{a.dp} reference done in {time.perf_counter() - t:.1f}s: {ref['loss']}", file=sys.stderr,
              flush=True)
    t = time.perf_counter()
    res = harness.run(_worker, a.pp * a.dp, env=env, timeout=a.timeout, pp=a.pp, virtual=a.virtual, **kw)
    last = res[a.pp - 1]  # the last stage of replica 0 holds the loss; every rank logs the global one
    out["pp"] = {k: last[k] for k in ("loss", "grad_norm", "step_s", "split", "engine")}
    out["pp"]["max_mem_gib_per_rank"] = [r["max_mem_gib"] for r in res]
    out["pp_wall_s"] = round(time.perf_counter() - t, 1)
    if not a.skip_ref:
        rl = max(abs(x - y) / max(1e-9, abs(y)) for x, y in zip(last["loss"], ref["loss"]))
        rg = max(abs(x - y) / max(1e-9, abs(y)) for x, y in zip(last["grad_norm"], ref["grad_norm"]))
        out["max_rel_diff"] = {"loss": rl, "grad_norm": rg}
        out["match"] = bool(rl < 1e-3 and rg < 1e-2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
