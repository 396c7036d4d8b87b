"""Host vs device time of eager and hipGraph-replayed training steps (distilgpt2 LoRA, bench shapes).

  python tools/graph_overhead.py [--steps 20]
Prints per mode: host issue time per step (time until train_step returns) and
device time per step (events), so launch-bound vs GPU-bound is visible.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mift import lora as L  # noqa: E402
from mift.data import MicroBatcher, synthetic_openwebtext  # noqa: E402
from mift.models import build_causal_lm  # noqa: E402
from mift.parallel import dist as D  # noqa: E402
from mift.train.trainer import TrainConfig, Trainer  # noqa: E402


def run(mode, steps, ctx):
    dev = ctx.device
    model = build_causal_lm("distilgpt2", dtype=torch.bfloat16, device=dev, seed=0)
    L.inject(model, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=["c_attn", "c_proj"]))
    ds = synthetic_openwebtext(32 * (steps + 5), 256, model.config.vocab_size, model.config.pad_token_id, seed=1)
    b = MicroBatcher(ds, 32, 1)
    tr = Trainer(model, b, TrainConfig(epochs=1, batch=32, accum=1, lr=5e-5, precision="bf16", logging_steps=0,
                                       save_steps=0, step_log="none", graph=mode), ctx)
    model.train()
    all_steps = list(b.epoch(0))
    for i in range(5):
        tr.train_step(all_steps[i])
    torch.cuda.synchronize()
    host = 0.0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for i in range(5, 5 + steps):
        h0 = time.perf_counter()
        tr.train_step(all_steps[i])
        host += time.perf_counter() - h0
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"{mode:5s} host_issue {host / steps * 1e3:.3f} ms/step  device {e0.elapsed_time(e1) / steps:.3f} ms/step  "
          f"wall {wall / steps * 1e3:.3f} ms/step", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    ctx = D.init(verbose=False, sanity=False)
    for mode in ("off", "on"):
        run(mode, a.steps, ctx)


if __name__ == "__main__":
    main()
