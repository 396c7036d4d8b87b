#!/usr/bin/env python
"""Flagship benchmark: distilgpt2 LoRA DDP fine-tuning throughput on MI355X
(``--model facebook/opt-2.7b [--pp S]``: the OPT LoRA pipeline-parallel configs).

Metric/config from BASELINE.json config #2: distilgpt2 LoRA (r=8, alpha=16,
dropout 0.05, targets c_attn,c_proj), bf16, seq_len 256, per-rank effective
batch 32 (reference batch 1 x accum 32, run as 32 x 1 — identical
token-normalised update), AdamW + clip 1.0 + linear LR, synthetic
OpenWebText-shaped tokens, random-init weights (no network).  One "step" =
one full optimizer step (forward, backward, gradient all-reduce over RCCL,
fused AdamW).  Weak scaling: every rank processes 32 x 256 tokens per step.

  python bench.py --gpus N --steps K --warmup W [--config {1..5}]

With N > 1 and no torchrun environment (WORLD_SIZE unset) this process starts the N ranks itself:
it runs ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1`` on this file
as a CHILD process (the parent never touches the GPU and never execs) and exits with its code.
Under torchrun (``WORLD_SIZE`` set, as the driver launches it) the formed world must equal
``--gpus``, else the run exits non-zero instead of silently measuring a different world.
``MIFT_BACKEND=gloo`` keeps the same command usable as an N-rank rehearsal on one GPU.

``--config`` selects a BASELINE.json config (recorded as ``config.config_id``):
  1  distilgpt2 LoRA DDP, world 1, CPU / gloo, fp32 (plumbing)
  2  distilgpt2 LoRA DDP bf16, 1..8 GPUs (default; the headline)
  3  OPT-2.7B fp16 LoRA, 4-stage pipeline (--gpus 4)
  4  OPT-2.7B fp16 LoRA, 2 DP x 4 PP (--gpus 8)
  5  OPT-6.7B fp16 LoRA, 8-stage pipeline (--gpus 8)

Prints ONE JSON line on rank 0.  `value` = whole-job steady-state tokens/s over the K timed
steps; ``wall_clock_epoch_s`` = one full epoch over a 20k-line medium_openwebtext-shaped
corpus (the reference's other metric, strong-scaled over the DP ranks) by a fresh model + Trainer,
timed from its first step like the reference's [Training] phase (its construction, incl. the
setup-time warm-up and graph capture, is reported as ``epoch.trainer_setup_s``; the same epoch on
the already-warm benchmark Trainer as ``epoch.warm_epoch_s``).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


# BASELINE.json "configs" -> bench presets (the reference's P1 / P2 shapes)
CONFIGS = {
    1: dict(model="distilgpt2", gpus=1, pp=1, precision="fp32", device="cpu", impl="torch",
            steps=2, warmup=1, epoch_lines=0),
    2: dict(model="distilgpt2", gpus=1, pp=1, precision="bf16"),
    3: dict(model="facebook/opt-2.7b", gpus=4, pp=4, precision="fp16"),
    4: dict(model="facebook/opt-2.7b", gpus=8, pp=4, precision="fp16"),
    5: dict(model="facebook/opt-6.7b", gpus=8, pp=8, precision="fp16"),
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default: the config's")
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS), help="BASELINE.json config id")
    ap.add_argument("--steps", type=int, default=None, help="timed optimizer steps (default 50)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed warmup steps (default 10)")
    ap.add_argument("--model", default=None)
    ap.add_argument("--device", default=None, choices=["gpu", "cpu"],
                    help="cpu: the world_size>=1 gloo/CPU plumbing path (config 1); default gpu")
    ap.add_argument("--seq_len", type=int, default=None, help="default 256 (GPT-2) / 512 (OPT, P2 sbatch)")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--accum", type=int, default=None, help="default 32 (P1) / 96 (P2 sbatch)")
    ap.add_argument("--fold_accum", type=int, default=1)
    ap.add_argument("--micro_batch", default="0",
                    help="regroup batch*accum into micro-batches of this size; 'auto' (PP default): "
                         "mift.parallel.plan's HBM-bounded cost model")
    ap.add_argument("--pp", type=int, default=None, help="pipeline stages (world = dp x pp)")
    ap.add_argument("--virtual_stages", dest="virtual", default=None,
                    help="interleaved 1F1B model chunks per pipeline rank; 'auto' (PP default): chosen with the "
                         "micro-batch by mift.parallel.plan")
    ap.add_argument("--partition", default=None, choices=["uniform", "balanced", "halves"],
                    help="pipeline split (default: halves for OPT — half-layer units —, else balanced)")
    ap.add_argument("--zero", type=int, default=0)
    ap.add_argument("--precision", default=None, choices=["bf16", "fp16", "fp32"],
                    help="default bf16 (GPT-2) / fp16 (OPT)")
    ap.add_argument("--impl", default=None, choices=["fused", "torch"],
                    help="fused = mift HIP kernels; torch = eager PyTorch ops on the same model (comparison)")
    ap.add_argument("--profile_dir", default=None, help="torch.profiler chrome trace of 3 steps")
    ap.add_argument("--epoch_lines", type=int, default=None,
                    help="after the timed steps, run one full epoch over this many medium_openwebtext-shaped "
                         "lines (README.md:66: ~20k) sharded over the DP ranks and report its wall clock "
                         "(the reference's [Training] sec metric, P1 and P2 alike: P2/summarize_opt_times.py:39-51); "
                         "default 20000, 0 skips it")
    a = ap.parse_args(argv)
    c = dict(CONFIGS[a.config])
    if a.model and a.model != c["model"]:  # a model override keeps that family's reference precision
        c["precision"] = "fp16" if "opt" in a.model.lower() else "bf16"
    a.model = a.model or c["model"]
    a.gpus = a.gpus if a.gpus is not None else c["gpus"]
    a.pp = a.pp if a.pp is not None else c["pp"]
    a.precision = a.precision or c["precision"]
    a.device = a.device or c.get("device", "gpu")
    a.impl = a.impl or c.get("impl", "torch" if a.device == "cpu" else "fused")
    a.steps = a.steps if a.steps is not None else c.get("steps", 50)
    a.warmup = a.warmup if a.warmup is not None else c.get("warmup", 10)
    if a.epoch_lines is None:
        a.epoch_lines = c.get("epoch_lines", 20000)
    if a.micro_batch == "0" and a.pp > 1:
        a.micro_batch = "auto"
    if a.virtual is None:
        a.virtual = "auto" if (a.pp > 1 and a.micro_batch == "auto") else "1"
    return a


def fail(msg, code=2):
    print(f"bench.py: error: {msg}", file=sys.stderr, flush=True)
    sys.exit(code)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(a):
    """Start the N ranks as a child ``torch.distributed.run`` (this process stays GPU-free: no HIP
    call, no exec) and return its exit code.  The worker ranks re-parse the same argv."""
    import subprocess
    if a.device != "cpu" and os.environ.get("MIFT_BACKEND", "nccl") != "gloo":
        import torch  # device_count() does not initialise HIP on this image
        have = torch.cuda.device_count()
        if have < a.gpus:
            fail(f"--gpus {a.gpus} needs {a.gpus} visible GPUs for one rank per GPU over RCCL, found {have} "
                 f"(MIFT_BACKEND=gloo rehearses N ranks on fewer GPUs; --device cpu runs the CPU path)")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 8) // (2 * a.gpus))))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench.py: launching {a.gpus} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main():
    a = parse_args()
    if a.gpus < 1 or a.gpus % a.pp:
        fail(f"--gpus {a.gpus} is not a multiple of the {a.pp} pipeline stages of config {a.config}")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch(a))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != a.gpus:
        fail(f"--gpus {a.gpus} but the launcher formed WORLD_SIZE={world_env}")
    if a.device == "cpu":
        os.environ["MIFT_DEVICE"] = "cpu"
    elif os.environ.get("MIFT_BACKEND", "nccl") != "gloo":
        import torch
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
        if torch.cuda.device_count() < lw:
            fail(f"{lw} local ranks need {lw} GPUs for RCCL, found {torch.cuda.device_count()}")
    # RCCL / Gloo print their init banners on fd 1 from native code; route
    # everything but the result line to stderr so stdout is exactly ONE JSON line.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    if a.impl == "torch":
        os.environ["MIFT_KERNELS"] = "0"
    import torch
    import torch.distributed as dist

    import mift
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.parallel import dist as D
    from mift.train.trainer import TrainConfig, Trainer

    is_opt = "opt" in a.model.lower()
    a.seq_len = a.seq_len or (512 if is_opt else 256)
    a.accum = a.accum or (96 if is_opt else 32)
    from mift.models.opt import OPTConfig
    from mift.models.gpt2 import GPT2Config
    mcfg = OPTConfig.preset(a.model) if is_opt else GPT2Config.preset(a.model)
    per_rank = a.batch * a.accum
    plan = None
    if a.pp > 1 and (a.micro_batch == "auto" or a.virtual == "auto"):
        # micro-batch and interleaving depth from the measured dp1 cost curve (before the grid is built:
        # interleaving needs the wrap-around links)
        from mift.parallel.plan import choose_micro_batch, stage_graphs_expected
        cands = None if a.micro_batch == "auto" else [int(a.micro_batch)]
        plan = choose_micro_batch(mcfg, a.seq_len, per_rank, a.pp, dtype_bytes=2, name=a.model, candidates=cands,
                                  virtual="auto" if a.virtual == "auto" else int(a.virtual),
                                  graphed=stage_graphs_expected(fused=a.impl == "fused" and a.device != "cpu"),
                                  partition=a.partition or ("halves" if is_opt else "balanced"))
        a.micro_batch, a.virtual = str(plan["micro_batch"]), str(plan["virtual"])
    V = int(a.virtual)
    ctx = D.init(pp=a.pp, verbose=False, sanity=True, virtual=V)
    n = ctx.world
    if n != a.gpus or ctx.pp != a.pp:
        fail(f"formed world {n} (pp {ctx.pp}) differs from --gpus {a.gpus} --pp {a.pp}")
    on_gpu = ctx.device.type == "cuda"
    if a.device == "gpu" and not on_gpu:
        fail("no GPU visible (use --device cpu / --config 1 for the CPU plumbing path)")
    if a.impl == "fused":
        if not on_gpu:
            fail("--impl fused needs a GPU")
        if not mift.kernels_available():
            fail(f"HIP extension not loaded: {mift._ext.error()!r}")
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.precision]

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    split = None
    kw = {}
    if ctx.pp > 1:
        from mift.parallel.pipeline import attn_cost_fraction, head_cost_layers, partition_layers, stage_chunks
        part = a.partition or ("halves" if is_opt else "balanced")
        split = partition_layers(mcfg.num_layers(), ctx.pp * V, part, head_cost_layers(mcfg), ranks=ctx.pp,
                                 attn_frac=attn_cost_fraction(mcfg))
        chunks = stage_chunks(split, ctx.pp, V, ctx.pp_rank)
        kw = dict(layer_range=chunks if V > 1 else chunks[0], has_embed=ctx.is_first_stage,
                  has_head=ctx.is_last_stage)
    model = build_causal_lm(a.model, dtype=dtype, device=ctx.device, seed=0, **kw)
    targets = ["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"] if is_opt else ["c_attn", "c_proj"]
    L.inject(model, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=targets,
                                 base_model_name_or_path=a.model))
    if a.impl == "torch":
        model.fused = False
    if a.micro_batch not in ("0", "auto") and per_rank % int(a.micro_batch) == 0:
        mb, acc = int(a.micro_batch), per_rank // int(a.micro_batch)
    else:
        mb, acc = (per_rank, 1) if (a.fold_accum and ctx.pp == 1) else (a.batch, a.accum)
    total_steps = a.warmup + a.steps
    ds = synthetic_openwebtext(per_rank * ctx.dp * total_steps, a.seq_len, model.config.vocab_size,
                               model.config.pad_token_id, seed=1234, full_length=True)
    batcher = MicroBatcher(ds, mb, acc, rank=ctx.dp_rank, world=ctx.dp)
    tr = Trainer(model, batcher, TrainConfig(epochs=1, batch=mb, accum=acc, lr=5e-5, precision=a.precision,
                                             logging_steps=0, save_steps=0, step_log="none", zero_stage=a.zero),
                 ctx)
    model.train()
    steps = list(batcher.epoch(0))
    assert len(steps) >= total_steps

    def run(i):
        tr.train_step(steps[i])

    for i in range(a.warmup):
        run(i)
    sync()
    if dist.is_initialized():
        dist.barrier()
    sync()
    trace = os.environ.get("MIFT_BENCH_TRACE") == "1"  # diagnostics: per-step host ms to stderr
    sync_every = int(os.environ.get("MIFT_BENCH_SYNC", "0"))  # diagnostics: host sync every k steps
    t0 = time.perf_counter()
    last = t0
    for i in range(a.warmup, total_steps):
        run(i)
        if not trace and ctx.rank == 0 and time.perf_counter() - last > 30.0:
            last = time.perf_counter()
            print(f"bench.py: step {i + 1 - a.warmup}/{a.steps} {last - t0:.1f}s", file=sys.stderr, flush=True)
        if trace or (sync_every and (i + 1) % sync_every == 0):
            sync()
        if trace:
            print(f"step {i} {(time.perf_counter() - t0) * 1000:.2f}", file=sys.stderr)
    sync()
    if dist.is_initialized():
        dist.barrier()
    sync()
    dt = time.perf_counter() - t0
    red_dev = ctx.device if ctx.backend == "nccl" else "cpu"
    t = torch.tensor([dt], dtype=torch.float64, device=red_dev)
    if dist.is_initialized() and n > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    ms = dt / a.steps * 1000.0
    tokens_per_step = per_rank * a.seq_len * ctx.dp
    value = tokens_per_step / (ms / 1000.0)
    stats = tr.opt.stats()
    if a.profile_dir and ctx.rank == 0:
        from torch.profiler import profile, ProfilerActivity
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for i in range(min(3, len(steps))):
                run(i % len(steps))
            sync()
        os.makedirs(a.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(a.profile_dir, "trace.json"))
        with open(os.path.join(a.profile_dir, "table.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))
    epoch_s, epoch_steps, warm_epoch_s, setup_s = None, None, None, None
    if a.epoch_lines > 0:
        # wall-clock/epoch, the other half of the BASELINE metric (reference: max over ranks of
        # `[Training] x sec`, P1/summarize_medium_times.py:4-10) over a medium-shaped corpus,
        # strong-scaled over the DP ranks like the reference's fixed dataset at N nodes.
        eds = synthetic_openwebtext(a.epoch_lines, a.seq_len, model.config.vocab_size, model.config.pad_token_id,
                                    seed=4321, full_length=True)

        def timed_epoch(trainer):
            eb_steps = list(MicroBatcher(eds, mb, acc, rank=ctx.dp_rank, world=ctx.dp).epoch(0))
            sync()
            if dist.is_initialized():
                dist.barrier()
            te = time.perf_counter()
            last = te
            for k, s_ in enumerate(eb_steps):
                trainer.train_step(s_)
                now = time.perf_counter()
                if now - last > 30.0 and ctx.rank == 0:  # progress (a silent multi-minute run looks hung)
                    print(f"bench.py: epoch step {k + 1}/{len(eb_steps)} {now - te:.1f}s", file=sys.stderr, flush=True)
                    last = now
            sync()
            if dist.is_initialized():
                dist.barrier()
            tt = torch.tensor([time.perf_counter() - te], dtype=torch.float64, device=red_dev)
            if dist.is_initialized() and n > 1:
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            return round(tt.item(), 4), len(eb_steps)

        # warm: the benchmark's own (already stepping) Trainer
        warm_epoch_s, _ = timed_epoch(tr)
        # cold: a FRESH model + Trainer as the P1 app builds them; [Training] is timed from its first
        # step (the reference definition), and its construction — which includes the setup-time
        # warm-up / graph capture (TrainConfig.warm_setup) — is reported separately as setup_s
        if tr.reducer is not None:
            tr.reducer.remove()
        del tr
        model2 = build_causal_lm(a.model, dtype=dtype, device=ctx.device, seed=0, **kw)
        L.inject(model2, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=targets,
                                      base_model_name_or_path=a.model))
        sync()
        ts = time.perf_counter()
        tr2 = Trainer(model2, MicroBatcher(eds, mb, acc, rank=ctx.dp_rank, world=ctx.dp),
                      TrainConfig(epochs=1, batch=mb, accum=acc, lr=5e-5, precision=a.precision, logging_steps=0,
                                  save_steps=0, step_log="none", zero_stage=a.zero), ctx)
        model2.train()
        sync()
        setup_s = round(time.perf_counter() - ts, 4)
        epoch_s, epoch_steps = timed_epoch(tr2)
    par = (f"dp{ctx.dp}" + (f"xpp{ctx.pp}" if ctx.pp > 1 else "") + (f"xv{V}" if V > 1 else "")
           + ("+zero1" if a.zero and ctx.dp > 1 else ""))
    # config_id only when the run IS that BASELINE config (model and pipeline depth); a --model / --pp
    # override is a custom run and says so instead of borrowing the default config's id
    base = CONFIGS[a.config]
    fam = lambda m: "opt" if "opt" in m.lower() else "gpt"  # noqa: E731
    config_id = a.config if (fam(a.model) == fam(base["model"]) and a.pp == base["pp"]) else None
    if ctx.rank == 0:
        kind = "PP" if ctx.pp > 1 else ("DDP" if ctx.dp > 1 or config_id is not None else "single-GPU")
        out = {
            "metric": ("" if config_id is not None else "custom config: ") +
                      f"{a.model.split('/')[-1]} LoRA {kind} fine-tune throughput (tokens/sec, whole job, "
                      f"steady state)",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.precision,
            "data": f"synthetic (OpenWebText-shaped random tokens, full {a.seq_len}-token lines); random-init weights",
            "config": {"model": a.model, "config_id": config_id, "global_batch": per_rank * ctx.dp,
                       "seq_len": a.seq_len, "backend": ctx.backend, "device": ctx.device.type,
                       "parallelism": par, "per_rank_batch": f"{a.batch}x{a.accum}", "micro_batch": f"{mb}x{acc}",
                       "split": split, "lora": "r8/a16/p0.05 " + ",".join(targets), "impl": a.impl,
                       "tokens_per_gpu_per_s": round(value / n, 1), "micro_batch_plan": plan,
                       "model_override": a.model != base["model"],
                       "final_grad_norm": round(stats["grad_norm"], 4)},
            "wall_clock_epoch_s": epoch_s,
            "epoch": {"lines": a.epoch_lines, "steps": epoch_steps, "global_batch": per_rank * ctx.dp,
                      "definition": "one pass over the medium-shaped corpus by a FRESH model + Trainer, timed "
                                    "from its first step, max over ranks (reference [Training] sec)",
                      "trainer_setup_s": setup_s,
                      "warm_epoch_s": warm_epoch_s}
            if epoch_s is not None else None,
        }
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    D.destroy()


if __name__ == "__main__":
    main()
