"""LoRA DDP fine-tuning application — the reference's W1 workload.

CLI-compatible with ``Cluster/Project 1 - Fine Tuning Distilgpt2/finetune_lora_distilgpt2.py:9-19``
(``--dataset --data_file --seq_len --epochs --batch --accum --lr --logdir --out_root``)
plus MI355X options (``--precision``, ``--fold_accum``, ``--synthetic``, ...).

Outputs (reference A.3): ``{logdir}/timing_rank{r}.log`` with the phases
Dataset load / Tokenization / Trainer setup / Training / Model save, and
``{out_root}/distilgpt2_lora_{dataset}_N{world}_{stamp}/`` holding the PEFT
adapter, the tokenizer files and ``run_meta.json`` (11 reference keys).
"""
import argparse
import datetime
import json
import os
import time

import torch

from .. import lora as L
from ..data import MicroBatcher, read_text_lines, synthetic_openwebtext, tokenize_lines, is_saved_dataset_dir, \
    load_pretokenized
from ..data.tokenizer import load_tokenizer
from ..models import build_causal_lm
from ..obs.timing import HOST, PhaseLogger
from ..parallel import dist as D
from ..train.trainer import TrainConfig, Trainer

DATASETS = {"tiny": "/data/tiny_openwebtext.txt", "medium": "/data/medium_openwebtext.txt"}
SYNTH_LINES = {"tiny": 2000, "medium": 20000}  # medium ≈ 20k lines (README.md:66)


def build_argparser(defaults=None):
    ap = argparse.ArgumentParser(description="mift LoRA DDP fine-tune (distilgpt2 reference CLI)")
    ap.add_argument("--dataset", choices=["tiny", "medium"], default="tiny")
    ap.add_argument("--data_file", type=str, default=None)
    ap.add_argument("--seq_len", type=int, default=256)
    ap.add_argument("--epochs", type=float, default=1)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--accum", type=int, default=32)
    ap.add_argument("--lr", type=float, default=5e-5)
    ap.add_argument("--logdir", type=str, default="logs")
    ap.add_argument("--out_root", type=str, default=os.path.expanduser("~/finetuned"))
    # mift extensions
    ap.add_argument("--model", type=str, default="distilgpt2")
    ap.add_argument("--base_weights", type=str, default=None, help="local HF checkpoint dir (else random init)")
    ap.add_argument("--tokenizer", type=str, default=None)
    ap.add_argument("--precision", choices=["bf16", "fp16", "fp32"], default=None)
    ap.add_argument("--fold_accum", type=int, default=-1,
                    help="run batch*accum as one micro-batch (identical token-normalised math); -1=auto(GPU)")
    ap.add_argument("--synthetic", type=int, default=-1, help="N synthetic lines (-1: only if data file missing)")
    ap.add_argument("--full_length", type=int, default=1)
    ap.add_argument("--lora_r", type=int, default=8)
    ap.add_argument("--lora_alpha", type=int, default=16)
    ap.add_argument("--lora_dropout", type=float, default=0.05)
    ap.add_argument("--target_modules", type=str, default=None)
    ap.add_argument("--max_steps", type=int, default=-1)
    ap.add_argument("--logging_steps", type=int, default=50)
    ap.add_argument("--save_steps", type=int, default=500)
    ap.add_argument("--resume", type=str, default=None)
    ap.add_argument("--gradient_checkpointing", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--step_log", choices=["p1", "lab", "none"], default="p1")
    ap.add_argument("--no_save", action="store_true")
    ap.add_argument("--profile", type=str, default=None,
                    help="dir: torch.profiler trace + kernel table + named-range ms per rank (mift.obs.profiler)")
    ap.add_argument("--profile_steps", type=str, default="3:6", help="global optimizer steps A:B (B exclusive)")
    ap.add_argument("--run_name", type=str, default=None, help="fixed run dir name (resume across jobs)")
    ap.add_argument("--config", type=str, default=None,
                    help="run config JSON (DeepSpeed keys + mift.* keys, mift.config.MiftConfig)")
    if defaults:
        ap.set_defaults(**defaults)
    return ap


def load_data(args, tok_vocab_pad, rank):
    """-> (TokenDataset, tokenizer, data_file_used)."""
    data_file = args.data_file or DATASETS[args.dataset]
    use_synth = args.synthetic > 0 or (args.synthetic < 0 and not os.path.exists(data_file))
    if use_synth:
        n = args.synthetic if args.synthetic > 0 else SYNTH_LINES[args.dataset]
        return ("synthetic", n, data_file)
    if is_saved_dataset_dir(data_file):
        return ("pretok", None, data_file)
    return ("text", read_text_lines(data_file), data_file)


def _write_job_meta(args, world, ctx):
    """``{logdir}/meta.json`` (reference P1 sbatch :72-87) unless the launcher already wrote one, so
    ``summarize_medium_times.py`` reports N and the dataset for app-only runs too."""
    path = os.path.join(args.logdir, "meta.json")
    if os.path.exists(path):
        return
    os.makedirs(args.logdir, exist_ok=True)
    meta = {"job_id": os.environ.get("SLURM_JOB_ID", os.path.basename(os.path.abspath(args.logdir))),
            "nnodes": int(os.environ.get("SLURM_NNODES", "1")), "world_size": world,
            "n_gpus": world if ctx.device.type == "cuda" else 0, "dataset": args.dataset,
            "data_file": args.data_file or DATASETS[args.dataset], "seq_len": args.seq_len, "epochs": args.epochs,
            "batch": args.batch, "accum": args.accum, "lr": args.lr, "model": args.model,
            "start": datetime.datetime.now().isoformat(timespec="seconds")}
    with open(path, "w") as f:
        json.dump(meta, f, indent=2)


def main(argv=None, defaults=None):
    args = build_argparser(defaults).parse_args(argv)
    torch.manual_seed(args.seed)
    from ..config import MiftConfig
    mcfg = MiftConfig.from_json(args.config)
    mcfg.apply_env()
    ctx = D.init()
    if ctx.rank == 0:
        for line in mcfg.report():
            print(line, flush=True)
    rank, world = ctx.rank, ctx.world
    gpu = ctx.device.type == "cuda"
    precision = args.precision or ("bf16" if gpu else "fp32")
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[precision]
    if not gpu and dtype != torch.float32:
        dtype = torch.float32  # CPU path keeps fp32 weights (autocast bf16 optional)
    logs = PhaseLogger(args.logdir, rank)
    if rank == 0:
        _write_job_meta(args, world, ctx)

    # --- Dataset load ---
    t0 = time.perf_counter()
    kind, payload, data_file = load_data(args, None, rank)
    logs.log("Dataset load", time.perf_counter() - t0)

    # --- Model / LoRA ---
    if rank == 0:
        print(f"[{HOST}] loading {args.model}", flush=True)
    model = build_causal_lm(args.model, dtype=dtype, device=ctx.device, seed=args.seed, weights=args.base_weights)
    vocab = model.config.vocab_size
    targets = args.target_modules.split(",") if args.target_modules else (
        ["c_attn", "c_proj"] if "gpt2" in args.model.lower() else ["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"])
    lcfg = L.LoraConfig(r=args.lora_r, lora_alpha=args.lora_alpha, lora_dropout=args.lora_dropout,
                        target_modules=targets, base_model_name_or_path=args.model)
    L.inject(model, lcfg, seed=args.seed)
    model.seed = args.seed

    # --- Tokenization ---
    t0 = time.perf_counter()
    tok = None
    if kind == "synthetic":
        pad = model.config.pad_token_id if hasattr(model.config, "pad_token_id") else vocab - 1
        ds = synthetic_openwebtext(payload, args.seq_len, vocab, pad, seed=1234, full_length=bool(args.full_length))
    elif kind == "pretok":
        ds = load_pretokenized(data_file, args.seq_len, model.config.pad_token_id, vocab)
    else:
        tok = load_tokenizer(args.tokenizer or args.model, corpus_lines=payload, vocab_size=vocab)
        ds = tokenize_lines(payload, tok, args.seq_len, tok.pad_id, vocab)
    logs.log("Tokenization", time.perf_counter() - t0)

    # --- Trainer setup ---
    t0 = time.perf_counter()
    fold = args.fold_accum if args.fold_accum >= 0 else int(gpu)
    mb, acc = (args.batch * args.accum, 1) if fold else (args.batch, args.accum)
    stamp = datetime.datetime.now().strftime("%Y%m%d-%H%M%S")
    base = args.model.split("/")[-1]
    # rank 0's clock names the run for everyone: per-rank stamps can straddle a second (or differ
    # across nodes) and then checkpoints / resume='auto' would use different directories per rank
    run_name = D.broadcast_obj(args.run_name or f"{base}_lora_{args.dataset}_N{world}_{stamp}")
    save_dir = os.path.join(args.out_root, run_name)
    batcher = MicroBatcher(ds, mb, acc, rank=ctx.dp_rank, world=ctx.dp, mode="strided")
    tcfg = TrainConfig(epochs=args.epochs, batch=mb, accum=acc, lr=args.lr, precision=precision,
                       logging_steps=args.logging_steps, save_steps=args.save_steps, max_steps=args.max_steps,
                       output_dir=save_dir, resume=args.resume,
                       recompute=bool(args.gradient_checkpointing) or mcfg.activation_checkpointing,
                       step_log=args.step_log, seed=args.seed, bucket_mb=mcfg.bucket_mb, graph=mcfg.graph,
                       consistency_every=mcfg.consistency_every, max_inflight_steps=mcfg.max_inflight_steps, max_grad_norm=mcfg.gradient_clipping,
                       weight_decay=mcfg.weight_decay, profile_dir=args.profile, profile_steps=args.profile_steps)
    trainer = Trainer(model, batcher, tcfg, ctx)
    logs.log("Trainer setup", time.perf_counter() - t0)

    # --- Train ---
    D.barrier()
    t0 = time.perf_counter()
    trainer.train()
    train_secs = time.perf_counter() - t0
    logs.log("Training", train_secs)
    D.barrier()

    # --- Save (rank 0) ---
    t0 = time.perf_counter()
    if rank == 0 and not args.no_save:
        os.makedirs(save_dir, exist_ok=True)
        L.save_pretrained(model, save_dir)
        if tok is not None:
            tok.save_pretrained(save_dir)
        meta = {"base_model": args.model, "world_size": world, "dataset": args.dataset, "data_file": data_file,
                "seq_len": args.seq_len, "epochs": args.epochs, "batch": args.batch, "accum": args.accum,
                "lr": args.lr, "host": HOST, "train_seconds": train_secs}
        with open(os.path.join(save_dir, "run_meta.json"), "w") as f:
            json.dump(meta, f, indent=2)
        print(f"✅ saved adapter + tokenizer to {save_dir}", flush=True)
    logs.log("Model save", time.perf_counter() - t0)
    # lines actually trained: whole epochs, or global_step full steps when --max_steps stops early
    lines = min(len(batcher.indices(0)) * args.epochs, trainer.global_step * batcher.mb * batcher.accum)
    tokens = lines * args.seq_len * ctx.dp
    if rank == 0:
        print(f"[RANK 0] TRAIN_RUNTIME_SEC={train_secs:.3f}", flush=True)
        print(f"[RANK 0] tokens_per_sec={tokens / max(train_secs, 1e-9):.1f} steps={trainer.global_step}", flush=True)
    D.destroy()
    return {"train_seconds": train_secs, "steps": trainer.global_step, "save_dir": save_dir,
            "history": trainer.history}


if __name__ == "__main__":
    main()
