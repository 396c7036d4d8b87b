"""Same-process A/B of whole training steps (distilgpt2 bench config, or OPT at micro-batch 12 x 512
fp16 with --model opt-2.7b; hipGraph replay).

Whole-process bench.py runs on one box differ by up to ~10 % from process to process, which
hides few-percent kernel changes.  Here two (or more) trainers are built in ONE process, each
under its own environment (kernel knobs are read when the step's graph is captured), and
their steps are timed in interleaved blocks; the medians are compared.

  python tools/step_ab.py "MIFT_GEMM_GROUP=0" "MIFT_GEMM_GROUP=4" [--blocks 6 --steps 10]
(AB_LORA_P=x / AB_MODEL_PDROP=x: diagnostic arms with other dropout rates)
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_env(spec):
    env = {}
    for kv in spec.split():
        k, _, v = kv.partition("=")
        env[k] = v
    return env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--model", default="distilgpt2")
    ap.add_argument("--mb", type=int, default=None, help="rows per step (default 32; OPT: 12 x 512 tokens)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.parallel import dist as D
    from mift.train.trainer import TrainConfig, Trainer

    ctx = D.init(verbose=False)
    opt = "opt" in a.model
    per_rank, seq = (a.mb or 12, 512) if opt else (a.mb or 32, 256)
    prec = "fp16" if opt else "bf16"
    targets = ["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"] if opt else ["c_attn", "c_proj"]
    trainers = []
    for spec in a.configs:
        env = parse_env(spec)
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        model = build_causal_lm(a.model, dtype=torch.float16 if opt else torch.bfloat16, device=ctx.device, seed=0)
        # diagnostics only: AB_LORA_P / AB_MODEL_PDROP change the dropout rates of this arm
        lp = float(env.get("AB_LORA_P", 0.05))
        if "AB_MODEL_PDROP" in env:
            for k in ("attn_pdrop", "resid_pdrop", "embd_pdrop"):
                setattr(model.config, k, float(env["AB_MODEL_PDROP"]))
        L.inject(model, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=lp, target_modules=targets,
                                     base_model_name_or_path=a.model))
        n = per_rank * (a.blocks * a.steps + 4)
        ds = synthetic_openwebtext(n, seq, model.config.vocab_size, model.config.pad_token_id, seed=1234,
                                   full_length=True)
        b = MicroBatcher(ds, per_rank, 1, rank=0, world=1)
        tr = Trainer(model, b, TrainConfig(epochs=1, batch=per_rank, accum=1, lr=5e-5, precision=prec,
                                           logging_steps=0, save_steps=0, step_log="none"), ctx)
        model.train()
        steps = list(b.epoch(0))
        for i in range(3):  # eager warm-up + capture + first replay, under this config's env
            tr.train_step(steps[i])
        torch.cuda.synchronize()
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        trainers.append((spec, tr, steps))
    ts = {spec: [] for spec, _, _ in trainers}
    for blk in range(a.blocks):
        order = trainers if blk % 2 == 0 else trainers[::-1]
        for spec, tr, steps in order:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i in range(a.steps):
                tr.train_step(steps[3 + (blk * a.steps + i) % (len(steps) - 3)])
            e.record()
            torch.cuda.synchronize()
            ts[spec].append(s.elapsed_time(e) / a.steps)
    out = {spec: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
                  "blocks": [round(x, 3) for x in v]} for spec, v in ts.items()}
    for spec, r in out.items():
        print(json.dumps({"config": spec, **r}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    D.destroy()


if __name__ == "__main__":
    main()
