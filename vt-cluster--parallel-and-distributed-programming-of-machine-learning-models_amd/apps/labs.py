"""The remaining course labs on the mift engine (SURVEY C16 lab variants, C28, C33).

* ``train_simple`` — `labs/simple_model/train_simple.py`: distilroberta-base
  sequence classification on AG-News, DDP, ``--dry_run`` (64 rows),
  ``max_steps=5``, ``logging_steps=1``, batch 8, lr 5e-5, rank banner and
  sample-batch shape lines, rank-0 save.
* ``fine_tune`` — `labs/fine_tuning/fine_tune.py`: FULL fine-tuning of a GPT-2
  causal LM (batch 2 x accum 4, lr 5e-5, max_length 128, ``--dry_run`` 64
  rows) on a text corpus (wikitext offline -> ``--data_file`` or a synthetic
  corpus), rank-0 save.
* ``transfer`` — `labs/transfer_learning/transfer.py`: distilbert-base-uncased
  + a fresh 2-way head on a sentiment corpus (IMDB offline -> a synthetic
  review corpus unless ``--data_file``), eval every epoch, rank-0 save.

All three use ``mift.train.Trainer(trainable="all")`` (flat fp32 arena, fused
AdamW, one gradient all-reduce per step over RCCL) and the HF-named models
of ``mift.models``; weights are random-init unless ``--weights`` names a
local HF checkpoint (no network), tokenizers come from ``--tokenizer`` or the
offline fallbacks of ``mift.data.agnews``.
"""
import argparse
import os
import socket

import numpy as np
import torch
import torch.distributed as dist

from ..data.agnews import TensorBatcher, encode, load_bert_tokenizer, load_split, HashWordTokenizer
from ..parallel import dist as D
from ..train.trainer import TrainConfig, Trainer


def _banner(ctx):
    print(f"[Rank {ctx.rank}/{ctx.world} | backend={ctx.backend}] PID={os.getpid()} on {socket.gethostname()}",
          flush=True)


def _tok(args, vocab):
    if args.tokenizer:
        from transformers import AutoTokenizer
        return AutoTokenizer.from_pretrained(args.tokenizer)
    # the BERT WordPiece vocab only for 30522-id models; otherwise hash words into the model's id space
    return load_bert_tokenizer() if vocab == 30522 else HashWordTokenizer(vocab)


def _common(ap):
    ap.add_argument("--local_rank", type=int, default=int(os.getenv("LOCAL_RANK", 0)))
    ap.add_argument("--dry_run", action="store_true")
    ap.add_argument("--weights", default=None)
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("--seed", type=int, default=42)
    return ap


def _train(model, data, batch, accum, lr, epochs, ctx, max_steps=-1, logging_steps=10, eval_fn=None):
    batcher = TensorBatcher(data, batch, rank=ctx.dp_rank, world=ctx.dp, shuffle=True, seed=42, drop_last=True)
    if accum > 1:
        batcher = _Accum(batcher, accum)
    tc = TrainConfig(epochs=epochs, batch=batch, accum=accum, lr=lr, precision="fp32", logging_steps=logging_steps,
                     step_log="none", save_steps=0, trainable="all", max_steps=max_steps, logging_first_step=True)
    tr = Trainer(model, batcher, tc, ctx, epoch_callbacks=[eval_fn] if eval_fn else ())
    return tr.train(), tr


class _Accum:
    """Group a TensorBatcher's micro-batches into optimizer steps of `accum`."""

    def __init__(self, b, accum):
        self.b, self.accum = b, accum

    def steps_per_epoch(self):
        return max(1, self.b.steps_per_epoch() // self.accum)

    def epoch(self, epoch=0, start_step=0):
        buf = []
        step = 0
        for mbs in self.b.epoch(epoch):
            buf += mbs
            if len(buf) == self.accum:
                if step >= start_step:
                    yield buf
                step += 1
                buf = []


# --------------------------------------------------------------- train_simple
def train_simple(argv=None):
    from ..models.encoders import build_classifier
    ap = _common(argparse.ArgumentParser(description="AG-News classification with data parallelism"))
    ap.add_argument("--model", default="distilroberta-base")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--output_dir", default="./model_output")
    ap.add_argument("--batch_size", type=int, default=8)
    ap.add_argument("--lr", type=float, default=5e-5)
    ap.add_argument("--max_steps", type=int, default=5)
    args, _ = ap.parse_known_args(argv)
    torch.manual_seed(args.seed)
    ctx = D.init(sanity=False, verbose=False)
    _banner(ctx)
    print(f"[Rank {ctx.rank}] Loading AG News dataset", flush=True)
    n = 64 if args.dry_run else 120000
    tr_t, tr_l, _ = load_split("train", 0, n, verbose=ctx.rank == 0)
    model = build_classifier(args.model, 4, device=ctx.device, seed=args.seed, weights=args.weights)
    print(f"[Rank {ctx.rank}] Tokenizing dataset", flush=True)
    tok = _tok(args, model.config.vocab_size)
    data = encode(tok, tr_t, tr_l, 128)
    print(f"[Rank {ctx.rank}] train size = {len(tr_l)}", flush=True)
    print(f"[Rank {ctx.rank}] Sample batch shapes: input_ids={tuple(data['input_ids'][:args.batch_size].shape)}, "
          f"labels={tuple(data['labels'][:args.batch_size].shape)}", flush=True)
    print(f"[Rank {ctx.rank}] Starting trainer.train()", flush=True)
    hist, _ = _train(model, data, args.batch_size, 1, args.lr, args.epochs, ctx, max_steps=args.max_steps,
                     logging_steps=1)
    print(f"[Rank {ctx.rank}] trainer.train() completed", flush=True)
    if ctx.rank == 0:
        print(f"[Rank {ctx.rank}] Saving model to {args.output_dir}", flush=True)
        model.save_pretrained(args.output_dir)
    D.destroy()
    return hist


# --------------------------------------------------------------- fine_tune
def _lm_corpus(args, n):
    if getattr(args, "data_file", None) and os.path.exists(args.data_file):
        from ..data import read_text_lines
        return [ln for ln in read_text_lines(args.data_file) if ln.strip()][:n]
    rng = np.random.default_rng(0)
    words = ("the of and to in a is was for on that with as by at from his her it an were are which this "
             "be has had also first one new after two years city team film season war").split()
    return [" ".join(rng.choice(words, size=int(rng.integers(20, 60)))) for _ in range(n)]


def fine_tune(argv=None):
    from ..data import lm_labels
    from ..models import build_causal_lm, save_hf_model
    ap = _common(argparse.ArgumentParser(description="Fine-tune a language model with parallelism"))
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--dataset", default="wikitext")
    ap.add_argument("--subset", default="wikitext-2-raw-v1")
    ap.add_argument("--data_file", default=None, help="offline corpus (one example per line)")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--batch_size", type=int, default=2)
    ap.add_argument("--output_dir", default="./finetuned")
    ap.add_argument("--max_steps", type=int, default=-1)
    args, _ = ap.parse_known_args(argv)
    torch.manual_seed(args.seed)
    ctx = D.init(sanity=False, verbose=False)
    _banner(ctx)
    lines = _lm_corpus(args, 64 if args.dry_run else 36718)
    model = build_causal_lm(args.model, device=ctx.device, seed=args.seed, weights=args.weights)
    model.fused = False  # full fine-tuning needs weight grads: the autograd path
    for p in model.parameters():
        p.requires_grad_(True)
    tok = HashWordTokenizer(model.config.vocab_size) if not args.tokenizer else _tok(args, model.config.vocab_size)
    enc = tok(lines, padding="max_length", truncation=True, max_length=128)
    ids = torch.as_tensor(np.asarray(enc["input_ids"]), dtype=torch.long)
    am = torch.as_tensor(np.asarray(enc["attention_mask"]), dtype=torch.long)
    pad = getattr(model.config, "pad_token_id", 0)
    data = {"input_ids": ids, "attention_mask": am, "labels": lm_labels(ids, am, pad)}
    hist, _ = _train(model, data, args.batch_size, 4, 5e-5, args.epochs, ctx, max_steps=args.max_steps)
    if ctx.rank == 0:
        save_hf_model(model, args.output_dir)
    D.destroy()
    return hist


# --------------------------------------------------------------- transfer
def _sentiment_corpus(n, seed):
    rng = np.random.default_rng(seed)
    pos = "great wonderful loved brilliant superb moving excellent fun beautiful best".split()
    neg = "awful boring hated terrible worst dull waste poor bad mess".split()
    neu = "the movie film plot actor scene story was it and this a of".split()
    texts, labels = [], []
    for _ in range(n):
        y = int(rng.integers(0, 2))
        w = [rng.choice(pos if y else neg) if rng.random() < 0.3 else rng.choice(neu) for _ in range(30)]
        texts.append(" ".join(w))
        labels.append(y)
    return texts, labels


def transfer(argv=None):
    from ..models.encoders import build_classifier
    ap = _common(argparse.ArgumentParser(description="Transfer learning example"))
    ap.add_argument("--base_model", default="distilbert-base-uncased")
    ap.add_argument("--dataset", default="imdb")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--output_dir", default="./transfer_model")
    args, _ = ap.parse_known_args(argv)
    torch.manual_seed(args.seed)
    ctx = D.init(sanity=False, verbose=False)
    _banner(ctx)
    n = 64 if args.dry_run else 25000
    tr_t, tr_l = _sentiment_corpus(n, 0)
    te_t, te_l = _sentiment_corpus(64 if args.dry_run else 2000, 1)
    model = build_classifier(args.base_model, 2, device=ctx.device, seed=args.seed, weights=args.weights)
    tok = _tok(args, model.config.vocab_size)
    train, test = encode(tok, tr_t, tr_l, 128), encode(tok, te_t, te_l, 128)
    accs = []

    def on_epoch(trainer, epoch):
        from .tiny_lab import evaluate
        acc = evaluate(model, test, ctx)
        accs.append(acc)
        if ctx.rank == 0:
            print(f"[RANK 0] epoch {epoch + 1} eval_accuracy={acc:.4f}", flush=True)

    hist, _ = _train(model, train, 8, 1, 5e-5, args.epochs, ctx, eval_fn=on_epoch)
    if ctx.rank == 0:
        model.save_pretrained(args.output_dir)
    D.destroy()
    return {"history": hist, "eval_accuracy": accs}
