"""One pipeline rank's compute, alone on one GPU.

Runs rank s of an S-stage (x V interleaved chunks) OPT pipeline through the PRODUCTION engine
(``PipelineEngine`` inside ``Trainer``: the exact ``schedule_1f1b`` / ``schedule_interleaved`` op list,
per-slot stage hipGraphs, the fused AdamW step) with every p2p replaced by a device-local exchange:
a receive copies a pre-filled random activation / gradient into its buffer (the bytes a real RCCL
receive would write), a send does nothing.  The measured time per optimizer step is the rank's
compute with no bubble and no transport; divided by the micro-batches per step it is the planner's
``stage_ms`` (parallel/plan.py ``predict``: max over ranks of the rank's per-micro-batch time), which
this tool checks for every rank of BASELINE configs 3 / 4 / 5:

  python tools/stage_time.py --config 3 [--micro_batch 12 --virtual 4] [--ranks 0,1,2,3] [--json out]

Each rank runs in its own child process (its own allocator, graphs and clocks), sequentially.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {3: ("facebook/opt-2.7b", 4, 1), 4: ("facebook/opt-2.7b", 4, 2), 5: ("facebook/opt-6.7b", 8, 1)}


class LocalP2P:
    """Stands in for ``parallel.comm.P2P``: receives are filled from a random pool, sends dropped."""

    def __init__(self, scale=1.0):
        self.pool, self.scale = {}, scale

    def post(self, sends=(), recvs=()):
        import torch
        from mift.parallel.comm import Pending
        out = []
        for t, _ in recvs:
            key = (tuple(t.shape), t.dtype, t.device)
            src = self.pool.get(key)
            if src is None:
                g = torch.Generator(device=t.device).manual_seed(7)
                src = self.pool[key] = (torch.randn(t.shape, device=t.device, generator=g) * self.scale).to(t.dtype)
            t.copy_(src, non_blocking=True)
            out.append(t)
        return Pending([], out, [], None)


def run_rank(model_name, S, V, s, mb, seq, per_replica, steps, warmup, precision="fp16", partition="balanced"):
    import torch
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.models.opt import OPTConfig
    from mift.parallel import dist as D
    from mift.parallel.pipeline import attn_cost_fraction, head_cost_layers, partition_layers, stage_chunks
    from mift.train.trainer import TrainConfig, Trainer

    ctx = D.init(pp=1, verbose=False, sanity=False)  # world 1; the grid below is simulated
    ctx.pp, ctx.pp_rank, ctx.pp_ranks, ctx.pp_virtual = S, s, list(range(S)), V
    cfg = OPTConfig.preset(model_name)
    split = partition_layers(cfg.num_hidden_layers, S * V, partition, head_cost_layers(cfg), ranks=S,
                             attn_frac=attn_cost_fraction(cfg))
    chunks = stage_chunks(split, S, V, s)
    dtype = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[precision]
    model = build_causal_lm(model_name, dtype=dtype, device=ctx.device, seed=0,
                            layer_range=chunks if V > 1 else chunks[0], has_embed=s == 0, has_head=s == S - 1)
    L.inject(model, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05,
                                 target_modules=["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"],
                                 base_model_name_or_path=model_name))
    acc = per_replica // mb
    ds = synthetic_openwebtext(per_replica * (warmup + steps), seq, cfg.vocab_size, cfg.pad_token_id, seed=1234,
                               full_length=True)
    batcher = MicroBatcher(ds, mb, acc)
    tr = Trainer(model, batcher, TrainConfig(epochs=1, batch=mb, accum=acc, lr=5e-5, precision=precision, logging_steps=0,
                                             save_steps=0, step_log="none"), ctx)
    eng = tr.engine
    act, grad = LocalP2P(1.0), LocalP2P(1e-3)
    for name in ("rx_f", "tx_f", "rx_wf", "tx_wf"):
        if hasattr(eng, name):
            setattr(eng, name, act)
    for name in ("rx_b", "tx_b", "rx_wb", "tx_wb"):
        if hasattr(eng, name):
            setattr(eng, name, grad)
    model.train()
    all_steps = list(batcher.epoch(0))
    for i in range(warmup):  # eager step, capture, first replays
        tr.train_step(all_steps[i])
    sync = torch.cuda.synchronize if ctx.device.type == "cuda" else (lambda: None)
    sync()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        tr.train_step(all_steps[i])
    sync()
    dt = (time.perf_counter() - t0) / steps
    out = {"rank": s, "chunks": [list(c) for c in chunks], "layers": sum(b - a for a, b in chunks),
           "partition": partition,
           "embed": s == 0, "head": s == S - 1, "micro_batch": mb, "micro_batches": acc,
           "ms_per_step": round(dt * 1e3, 2), "ms_per_micro_batch": round(dt * 1e3 / acc, 3),
           "replays": eng.stats.get("replays", 0), "split": split,
           "peak_gib": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2) if ctx.device.type == "cuda" else 0.0}
    D.destroy()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--micro_batch", type=int, default=None, help="default: the planner's choice")
    ap.add_argument("--virtual", type=int, default=None, help="default: the planner's choice")
    ap.add_argument("--seq_len", type=int, default=512)
    ap.add_argument("--per_replica", type=int, default=96)
    ap.add_argument("--ranks", default=None)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--json", default=None)
    ap.add_argument("--model", default=None, help="override the config's model (e.g. opt-tiny for a CPU check)")
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--pp", type=int, default=None, help="override the config's stage count")
    ap.add_argument("--partition", default="balanced", choices=["uniform", "balanced", "halves"])
    ap.add_argument("--child", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child is not None:
        kw = json.loads(a.child)
        print("RESULT " + json.dumps(run_rank(**kw)), flush=True)
        return
    from mift.models.opt import OPTConfig
    from mift.parallel.plan import choose_micro_batch, predict
    name, S, dp = CONFIGS[a.config]
    name = a.model or name
    S = a.pp or S
    cfg = OPTConfig.preset(name)
    plan = choose_micro_batch(cfg, a.seq_len, a.per_replica, S, name=name,
                              candidates=[a.micro_batch] if a.micro_batch else None,
                              virtual=a.virtual if a.virtual else "auto", partition=a.partition)
    mb, V = plan["micro_batch"], plan["virtual"]
    pred = predict(cfg, a.seq_len, a.per_replica, S, mb, name=name, virtual=V, partition=a.partition)
    ranks = [int(r) for r in a.ranks.split(",")] if a.ranks else list(range(S))
    rows = []
    for s in ranks:
        kw = dict(model_name=name, S=S, V=V, s=s, mb=mb, seq=a.seq_len, per_replica=a.per_replica,
                  steps=a.steps, warmup=a.warmup, precision=a.precision, partition=a.partition)
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", json.dumps(kw)],
                           capture_output=True, text=True, cwd=ROOT)
        res = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
        if p.returncode != 0 or not res:
            print(p.stdout[-2000:], p.stderr[-4000:], file=sys.stderr)
            sys.exit(p.returncode or 1)
        r = json.loads(res[0][7:])
        rows.append(r)
        print(json.dumps(r), flush=True)
    worst = max(r["ms_per_micro_batch"] for r in rows)
    summary = {"config": a.config, "model": name, "stages": S, "dp": dp, "virtual": V, "micro_batch": mb,
               "partition": a.partition,
               "pred_stage_ms": pred["stage_ms"], "meas_stage_ms": worst,
               "meas_over_pred": round(worst / pred["stage_ms"], 3), "pred_step_ms": pred["step_ms"],
               "per_rank_ms_per_micro_batch": [r["ms_per_micro_batch"] for r in rows],
               "bubble_free_step_ms": round(worst * rows[0]["micro_batches"], 2),
               "slowest_over_mean": round(worst / (sum(r["ms_per_micro_batch"] for r in rows) / len(rows)), 3)}
    print("SUMMARY " + json.dumps(summary), flush=True)
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump({"summary": summary, "ranks": rows, "plan": plan}, f, indent=1)


if __name__ == "__main__":
    main()
