"""OPT LoRA fine-tuning with pipeline parallelism (+ optional DP and ZeRO-1) —
the reference's W2 workload.

CLI-compatible with ``Cluster/Project 2 - Course Project/finetune_lora_opt_pp.py:24-36``
(``--model_name --data_file --seq_len --epochs --batch --accum --lr --logdir
--out_root --ds_cfg``, unknown args ignored like ``parse_known_args``) and the
launch env (``RANK/WORLD_SIZE/LOCAL_RANK`` with SLURM fallbacks,
``PIPELINE_PARALLEL_SIZE`` defaulting to the world size, `:38-54`).

``--ds_cfg`` accepts the DeepSpeed JSON the reference ships
(`deepspeed_pp_zero1_cpu_activ.json`): ``train_micro_batch_size_per_gpu``,
``zero_optimization.stage``, ``fp16/bf16.enabled``, ``optimizer.params``
(betas, eps, weight_decay) and ``gradient_clipping`` are honoured; as in the
reference, ``--accum`` and ``--lr`` from the CLI win (``engine.set_lr`` /
``set_gradient_accumulation_steps``, `:207-208`).  The JSON is parsed into the
typed ``mift.config.MiftConfig`` (which also reads the ``mift.*`` MI355X keys):
keys that only make sense for DeepSpeed-on-CPU (``cpu_offload``,
``partition_activations``, ``cpu_checkpointing``) are accepted without effect and
REPORTED at start-up (288 GB of HBM per GPU holds every stage's weights and
in-flight activations); unknown keys are an error.

Outputs: P2 loss lines ``[R{r}] ep=.. step=.. loss=.. (+..s)`` from the last
stage every 10 steps (`:219-224`), ``{logdir}/timing_rank{r}.log`` phases, and
on rank 0 ``{out_root}/opt27b_lora_pp_{unix}/`` with the FULL PEFT adapter
(gathered from all stages — the reference would have saved only stage 0's
view), the tokenizer, and ``meta.json`` ``{"split": [...], "stages": S}``.
"""
import argparse
import json
import os
import time

import torch

from .. import lora as L
from ..data import MicroBatcher, is_saved_dataset_dir, load_pretokenized, read_text_lines, synthetic_openwebtext, \
    tokenize_lines
from ..data.tokenizer import load_tokenizer
from ..models import build_causal_lm
from ..obs.timing import PhaseLogger, p2_loss_line
from ..parallel import dist as D
from ..parallel.pipeline import attn_cost_fraction, head_cost_layers, partition_layers, stage_chunks, stage_layer_range
from ..train.trainer import TrainConfig, Trainer


def build_argparser():
    ap = argparse.ArgumentParser(description="mift LoRA fine-tune of OPT with pipeline parallelism")
    ap.add_argument("--model_name", default="facebook/opt-2.7b")
    ap.add_argument("--data_file", required=True, help="plain-text file (one example per line) or saved dataset dir")
    ap.add_argument("--seq_len", type=int, default=1024)
    ap.add_argument("--epochs", type=float, default=1)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--accum", type=int, default=64)
    ap.add_argument("--lr", type=float, default=5e-5)
    ap.add_argument("--logdir", default="logs")
    ap.add_argument("--out_root", default=os.path.expanduser("~/finetuned"))
    ap.add_argument("--ds_cfg", default="deepspeed_pp_zero1_cpu.json")
    # mift extensions
    ap.add_argument("--pp", type=int, default=None, help="pipeline stages (default $PIPELINE_PARALLEL_SIZE or world)")
    ap.add_argument("--virtual_stages", default=None,
                    help="interleaved 1F1B: model chunks per pipeline rank, or 'auto' (chosen with the micro-batch "
                         "by the planner); default $PIPELINE_VIRTUAL_STAGES, mift.virtual_stages, else 'auto' when "
                         "the micro-batch is planned and 1 otherwise")
    ap.add_argument("--partition", choices=["uniform", "balanced", "halves"], default=None,
                    help="layer split (default: mift.pp_partition / pipeline.partition_method, else balanced; "
                         "halves: half-layer units, a stage boundary may split a decoder layer between its "
                         "attention and MLP sub-blocks)")
    ap.add_argument("--precision", choices=["fp16", "bf16", "fp32"], default=None)
    ap.add_argument("--micro_batch", default=None,
                    help="GPU micro-batch: regroups batch*accum sequences per step into micro-batches of this "
                         "size (same token-normalised update, fewer pipeline bubbles); 'auto' = the planner "
                         "(mift.parallel.plan, measured dp1 cost curve + HBM bound; the default on GPU with "
                         ">1 stage, or mift.micro_batch); 0 = keep the DeepSpeed / --batch micro-batch")
    ap.add_argument("--zero", type=int, default=None, help="ZeRO stage override (0/1)")
    ap.add_argument("--synthetic", type=int, default=-1, help="N synthetic lines (-1: only if data file missing)")
    ap.add_argument("--base_weights", default=None)
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("--lora_r", type=int, default=8)
    ap.add_argument("--lora_alpha", type=int, default=16)
    ap.add_argument("--lora_dropout", type=float, default=0.05)
    ap.add_argument("--target_modules", default="q_proj,k_proj,v_proj,out_proj,fc1,fc2")
    ap.add_argument("--max_steps", type=int, default=-1)
    ap.add_argument("--profile", type=str, default=None,
                    help="dir: torch.profiler trace + kernel table + named-range ms per rank (mift.obs.profiler)")
    ap.add_argument("--profile_steps", type=str, default="3:6", help="global optimizer steps A:B (B exclusive)")
    ap.add_argument("--log_every", type=int, default=10)
    ap.add_argument("--gradient_checkpointing", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--save_steps", type=int, default=0)
    ap.add_argument("--resume", default=None)
    ap.add_argument("--no_save", action="store_true")
    return ap


def read_ds_config(path):
    """DeepSpeed JSON (+ ``mift.*`` keys) -> mift.config.MiftConfig (missing file -> inline defaults)."""
    from ..config import MiftConfig
    return MiftConfig.from_json(path)


def _will_use_gpu():
    if os.environ.get("MIFT_DEVICE", "") == "cpu":
        return False
    return torch.cuda.device_count() > 0  # counting devices does not initialise HIP


def plan_micro_batch(args, ds, stages, world, gpu):
    """Resolve (GPU micro-batch, virtual stages, plan) before the process grid is built (interleaving
    needs the wrap-around links).  The reference CLI (``--batch 1 --accum 96``) on a GPU pipeline runs
    the planner's micro-batch: micro-batch 1 leaves MI355X's matrix cores idle (OPT-2.7B 25.5 ms per
    sequence at mb 1 vs 6.8 at mb 12, parallel/plan.py MEASURED) — the token-normalised update is the
    same for any regrouping of the batch*accum sequences of a step."""
    mbsel = args.micro_batch if args.micro_batch is not None else ds.micro_batch
    if mbsel in (0, "0", None) and args.micro_batch is None and gpu and stages > 1:
        mbsel = "auto"
    mbsel = "auto" if str(mbsel).lower() == "auto" else int(mbsel or 0)
    vsel = args.virtual_stages or os.environ.get("PIPELINE_VIRTUAL_STAGES") or ds.virtual_stages
    if vsel is None:
        vsel = "auto" if mbsel == "auto" else 1
    vsel = "auto" if str(vsel).lower() == "auto" else int(vsel)
    base_mb = ds.micro_batch_size or args.batch
    per_step = base_mb * args.accum          # sequences per optimizer step per DP replica
    plan = None
    if stages > 1 and (mbsel == "auto" or vsel == "auto"):
        from ..models.opt import OPTConfig
        from ..parallel.plan import choose_micro_batch, stage_graphs_expected
        cfg = OPTConfig.preset(args.model_name)
        rec = bool(getattr(args, "gradient_checkpointing", False)) or bool(getattr(ds, "activation_checkpointing", False))
        plan = choose_micro_batch(cfg, args.seq_len, per_step, stages, dtype_bytes=2, name=args.model_name,
                                  candidates=None if mbsel == "auto" else [mbsel or base_mb],
                                  virtual=vsel, graphed=stage_graphs_expected(recompute=rec),
                                  partition=args.partition or ds.pp_partition)
        mbsel, vsel = plan["micro_batch"], plan["virtual"]
    elif mbsel == "auto":
        mbsel = 0
    if vsel == "auto":
        vsel = 1
    return (mbsel or 0), int(vsel), plan


def main(argv=None):
    args, _unknown = build_argparser().parse_known_args(argv)
    world_env = int(os.environ.get("WORLD_SIZE", os.environ.get("SLURM_NTASKS", "1")))
    stages = args.pp or int(os.environ.get("PIPELINE_PARALLEL_SIZE", str(world_env)))
    assert 1 <= stages <= 32, "PIPELINE_PARALLEL_SIZE must be in [1,32]"
    ds = read_ds_config(args.ds_cfg)
    gmb, virtual, plan = plan_micro_batch(args, ds, stages, world_env, _will_use_gpu())
    ctx = D.init(pp=stages, virtual=virtual)
    rank = ctx.rank

    def log(msg):
        print(f"[R{rank}] {msg}", flush=True)

    gpu = ctx.device.type == "cuda"
    ds.apply_env()
    if rank == 0:
        for line in ds.report():
            print(line, flush=True)
        if plan is not None:
            print(f"[R0] micro-batch plan: mb={plan['micro_batch']} virtual={plan['virtual']} "
                  f"predicted step {plan['step_ms']} ms, per-GPU efficiency vs dp1 {plan['efficiency_vs_dp1']}, "
                  f"activations {plan['act_gib']} GiB", flush=True)
    precision = args.precision or ("fp32" if not gpu else ("bf16" if ds.bf16 else "fp16"))
    if not gpu:
        precision = "fp32"
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[precision]
    zero = args.zero if args.zero is not None else ds.zero_stage
    logs = PhaseLogger(args.logdir, rank)

    # ---- data (every stage of a replica reads the same shard: DP rank, not global rank) ----
    t0 = time.perf_counter()
    use_synth = args.synthetic > 0 or (args.synthetic < 0 and not os.path.exists(args.data_file))
    if use_synth:
        log(f"Data file {args.data_file} not found: synthetic OpenWebText-shaped lines")
    elif is_saved_dataset_dir(args.data_file):
        log(f"Loading pre-tokenized dataset from disk: {args.data_file}")
    else:
        log(f"Loading RAW text file: {args.data_file}")
    lines = None if (use_synth or is_saved_dataset_dir(args.data_file)) else read_text_lines(args.data_file)
    logs.log("Dataset load", time.perf_counter() - t0, echo=False)

    # ---- stage model: only this stage's layers are ever allocated ----
    t0 = time.perf_counter()
    from ..models.opt import OPTConfig
    cfg = OPTConfig.preset(args.model_name)
    N = cfg.num_hidden_layers
    V = ctx.pp_virtual
    split = partition_layers(N, ctx.pp * V, args.partition or ds.pp_partition, head_cost_layers(cfg), ranks=ctx.pp,
                             attn_frac=attn_cost_fraction(cfg))
    mine = stage_chunks(split, ctx.pp, V, ctx.pp_rank)  # V == 1: one contiguous range
    lo, hi = mine[0][0], mine[-1][1]
    model = build_causal_lm(args.model_name, dtype=dtype, device=ctx.device, seed=args.seed,
                            weights=args.base_weights, layer_range=mine if V > 1 else mine[0],
                            has_embed=ctx.is_first_stage, has_head=ctx.is_last_stage)
    lcfg = L.LoraConfig(r=args.lora_r, lora_alpha=args.lora_alpha, lora_dropout=args.lora_dropout,
                        target_modules=args.target_modules.split(","), base_model_name_or_path=args.model_name)
    L.inject(model, lcfg, seed=args.seed)
    model.seed = args.seed
    log(f"Pipeline split={split} (total blocks={N}, stages={ctx.pp}"
        + (f", {V} interleaved chunks per stage) -> my chunks {mine}" if V > 1 else f") -> my layers [{lo},{hi})"))
    logs.log("Model build", time.perf_counter() - t0, echo=False)

    # ---- tokenization ----
    t0 = time.perf_counter()
    tok = None
    if use_synth:
        n = args.synthetic if args.synthetic > 0 else 4096
        data = synthetic_openwebtext(n, args.seq_len, cfg.vocab_size, cfg.pad_token_id, seed=1234)
    elif lines is None:
        data = load_pretokenized(args.data_file, args.seq_len, cfg.pad_token_id, cfg.vocab_size)
        log("Detected tokenized dataset")
    else:
        tok = load_tokenizer(args.tokenizer or args.model_name, corpus_lines=lines, vocab_size=cfg.vocab_size)
        log(f"Detected raw text; tokenizing (seq_len={args.seq_len})")
        data = tokenize_lines(lines, tok, args.seq_len, cfg.pad_token_id, cfg.vocab_size)
    logs.log("Tokenization", time.perf_counter() - t0, echo=False)

    # ---- engine ----
    t0 = time.perf_counter()
    mb = ds.micro_batch_size or args.batch
    per_step = mb * args.accum
    if gmb and per_step % gmb == 0:
        mb = gmb
    accum = per_step // mb
    batcher = MicroBatcher(data, mb, accum, rank=ctx.dp_rank, world=ctx.dp)
    tcfg = TrainConfig(epochs=args.epochs, batch=mb, accum=accum, lr=args.lr, precision=precision,
                       weight_decay=ds.weight_decay, max_grad_norm=ds.gradient_clipping, logging_steps=args.log_every,
                       step_log="none", max_steps=args.max_steps, seed=args.seed, zero_stage=zero,
                       recompute=bool(args.gradient_checkpointing) or ds.activation_checkpointing,
                       bucket_mb=ds.bucket_mb, graph=ds.graph, consistency_every=ds.consistency_every, max_inflight_steps=ds.max_inflight_steps,
                       save_steps=args.save_steps,
                       output_dir=os.path.join(args.out_root, "checkpoints") if args.save_steps else None,
                       resume=args.resume, profile_dir=args.profile, profile_steps=args.profile_steps)
    t_last = [time.perf_counter()]

    def p2_log(trainer, rec):
        if ctx.is_last_stage and ctx.dp_rank == 0:
            now = time.perf_counter()
            ep = int((trainer.global_step - 1) // max(1, trainer.steps_per_epoch))
            print(p2_loss_line(rank, ep, trainer.global_step - 1, rec["loss"], now - t_last[0]), flush=True)
            t_last[0] = now

    trainer = Trainer(model, batcher, tcfg, ctx, callbacks=[p2_log])
    log(f"engine initialized (stage {ctx.pp_rank}/{ctx.pp}, dp {ctx.dp_rank}/{ctx.dp}, mb={mb}x{accum}, "
        f"{precision}, zero={zero})")
    logs.log("Trainer setup", time.perf_counter() - t0, echo=False)

    D.barrier()
    t0 = time.perf_counter()
    trainer.train()
    if gpu:
        torch.cuda.synchronize()
    train_secs = time.perf_counter() - t0
    logs.log("Training", train_secs)
    D.barrier()

    t0 = time.perf_counter()
    state = trainer.adapter_state()
    out = None
    if rank == 0 and not args.no_save:
        out = os.path.join(args.out_root, f"opt27b_lora_pp_{int(time.time())}")
        L.save_adapter(out, state, lcfg)
        if tok is not None:
            tok.save_pretrained(out)
        with open(os.path.join(out, "meta.json"), "w") as f:
            json.dump({"split": split, "stages": ctx.pp, "virtual_stages": ctx.pp_virtual, "micro_batch": mb,
                       "micro_batches_per_step": accum, "micro_batch_plan": plan}, f, indent=2)
        log(f"Saved adapters+tokenizer to {out}")
    logs.log("Model save", time.perf_counter() - t0, echo=False)
    tokens = trainer.global_step * per_step * args.seq_len * ctx.dp
    if rank == 0:
        print(f"[R0] TRAIN_RUNTIME_SEC={train_secs:.3f} tokens_per_sec={tokens / max(train_secs, 1e-9):.1f} "
              f"steps={trainer.global_step}", flush=True)
    D.destroy()
    return {"train_seconds": train_secs, "steps": trainer.global_step, "save_dir": out, "split": split,
            "history": trainer.history, "micro_batch": mb, "virtual_stages": ctx.pp_virtual, "plan": plan}


if __name__ == "__main__":
    main()
