"""The tiny-BERT AG-News lab (W3): DDP training, DDP inference, accuracy check.

CLIs and log lines follow the reference lab scripts so ``eval_logs.py``-style
parsers and the submission greps keep working:

* ``train``  — `labs/tiny/train_tiny.py:108-203`: ``--epochs 3 --subset 2000
  --batch 16 --out ./tiny_out``; prints ``[RANK r] WORLD_SIZE=w``, per-step
  ``[rank r | step N] step_ms=.. samples_per_sec=.. tokens_per_sec=..``,
  per-log ``[rank r | step N] loss=..`` (+ ``log.rank{r}.txt`` and TensorBoard
  scalars under ``out/tb/rank{r}``), ``[RANK 0] TRAIN_RUNTIME_SEC=..``, an
  eval every epoch on ALL ranks and ``[RANK 0] EVAL accuracy=..``; rank 0 saves
  model + tokenizer to ``--out``.  Hyper-parameters of the reference
  ``TrainingArguments``: lr 5e-4, AdamW, linear decay, clip 1.0, seed 42.
* ``infer``  — `labs/tiny/infer_ddp.py`: round-robin shard of test[:max_test],
  local counts → SUM all-reduce, time → MAX, and
  ``[RANK 0] INFER global_accuracy=.. global_samples_per_sec=.. global_tokens_per_sec=..``.
* ``test``   — `labs/tiny/test_tiny.py`: accuracy on test[:512] + 3 example predictions.

MI355X: one process per GPU over RCCL; the 0.5 M-parameter model trains all
weights (flat fp32 arena + fused AdamW, one gradient all-reduce per step).
"""
import argparse
import os
import random
import time

import torch
import torch.distributed as dist

from ..data.agnews import LABELS, TensorBatcher, encode, load_bert_tokenizer, load_split
from ..models.bert import BertConfig, BertForSequenceClassification
from ..obs.tb import PerRankLogger
from ..parallel import dist as D
from ..train.trainer import TrainConfig, Trainer

SEQ = 128


@torch.no_grad()
def evaluate(model, data, ctx, batch=64):
    """Global accuracy of ``model`` on ``data`` (round-robin DP shard, SUM all-reduce)."""
    model.eval()
    n = len(data["labels"])
    idx = list(range(n))[ctx.dp_rank::ctx.dp]
    corr = tot = 0
    for i in range(0, len(idx), batch):
        j = torch.as_tensor(idx[i:i + batch])
        ids = data["input_ids"][j].to(ctx.device)
        am = data["attention_mask"][j].to(ctx.device)
        pred = model(input_ids=ids, attention_mask=am)["logits"].argmax(-1).cpu()
        corr += int((pred == data["labels"][j]).sum())
        tot += len(j)
    t = torch.tensor([corr, tot], dtype=torch.float64)
    if ctx.world > 1:
        dist.all_reduce(t, group=ctx.ctrl_group)
    model.train()
    return t[0].item() / max(1.0, t[1].item())


def train(argv=None):
    p = argparse.ArgumentParser(description="tiny BERT AG-News DDP training")
    p.add_argument("--epochs", type=int, default=3)
    p.add_argument("--subset", type=int, default=2000)
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--out", default="./tiny_out")
    p.add_argument("--local_rank", type=int, default=int(os.getenv("LOCAL_RANK", 0)))
    p.add_argument("--lr", type=float, default=5e-4)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--eval_rows", type=int, default=512)
    p.add_argument("--no_tb", action="store_true")
    args, _ = p.parse_known_args(argv)
    torch.manual_seed(args.seed)
    ctx = D.init(sanity=False)
    tok = load_bert_tokenizer()
    tr_txt, tr_lab, _ = load_split("train", 0, args.subset, verbose=ctx.rank == 0)
    te_txt, te_lab, _ = load_split("test", 0, args.eval_rows, verbose=ctx.rank == 0)
    train_data, test_data = encode(tok, tr_txt, tr_lab, SEQ), encode(tok, te_txt, te_lab, SEQ)
    vocab = getattr(tok, "vocab_size", 30522)
    model = BertForSequenceClassification(BertConfig.tiny(vocab, len(LABELS)), device=ctx.device)
    model.init_weights(args.seed)
    batcher = TensorBatcher(train_data, args.batch, rank=ctx.dp_rank, world=ctx.dp, shuffle=True, seed=args.seed)
    tc = TrainConfig(epochs=args.epochs, batch=args.batch, accum=1, lr=args.lr, precision="fp32", logging_steps=10,
                     logging_first_step=True, step_log="lab", save_steps=0, trainable="all", seed=args.seed)
    rlog = PerRankLogger(args.out, ctx.rank, use_tb=not args.no_tb)

    def on_log(trainer, rec):
        rlog.log(trainer.global_step, rec)

    def on_epoch(trainer, epoch):
        acc = evaluate(model, test_data, ctx)
        rlog.log(trainer.global_step, {"eval_accuracy": round(acc, 4), "epoch": epoch + 1})

    trainer = Trainer(model, batcher, tc, ctx, callbacks=[on_log], epoch_callbacks=[on_epoch])
    t0 = time.perf_counter()
    trainer.train()
    t1 = time.perf_counter()
    if ctx.rank == 0:
        print(f"[RANK 0] TRAIN_RUNTIME_SEC={t1 - t0:.3f}", flush=True)
    acc = evaluate(model, test_data, ctx)  # on ALL ranks (elastic exit-barrier race, train_tiny.py:188)
    if ctx.rank == 0:
        print(f"[RANK 0] EVAL accuracy={acc:.4f}", flush=True)
    D.barrier()
    if ctx.rank == 0:
        model.save_pretrained(args.out)
        tok.save_pretrained(args.out)
    rlog.close()
    D.destroy()
    return {"train_seconds": t1 - t0, "accuracy": acc}


def _load_ckpt(path, device):
    return BertForSequenceClassification.from_pretrained(path, device=device).eval(), load_bert_tokenizer(path)


def infer(argv=None):
    p = argparse.ArgumentParser(description="tiny BERT DDP inference")
    p.add_argument("--ckpt", required=True)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--max_test", type=int, default=2048)
    p.add_argument("--seq_len", type=int, default=128)
    p.add_argument("--local_rank", type=int, default=int(os.getenv("LOCAL_RANK", 0)))
    args, _ = p.parse_known_args(argv)
    ctx = D.init(sanity=False)
    model, tok = _load_ckpt(args.ckpt, ctx.device)
    txt, lab, _ = load_split("test", 0, args.max_test, verbose=ctx.rank == 0)
    data = encode(tok, txt, lab, args.seq_len)
    idx = list(range(len(lab)))[ctx.rank::ctx.world]
    corr = tot = toks = 0
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.inference_mode():
        for i in range(0, len(idx), args.batch):
            j = torch.as_tensor(idx[i:i + args.batch])
            logits = model(input_ids=data["input_ids"][j].to(ctx.device),
                           attention_mask=data["attention_mask"][j].to(ctx.device))["logits"]
            pred = logits.argmax(-1).cpu()
            corr += int((pred == data["labels"][j]).sum())
            tot += len(j)
            toks += len(j) * args.seq_len
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sums = torch.tensor([corr, tot, toks], dtype=torch.float64)
    tmax = torch.tensor([dt], dtype=torch.float64)
    if ctx.world > 1:
        dist.all_reduce(sums, group=ctx.ctrl_group)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX, group=ctx.ctrl_group)
    acc = sums[0].item() / max(1.0, sums[1].item())
    wall = max(1e-9, tmax.item())
    if ctx.rank == 0:
        print(f"[RANK 0] INFER global_accuracy={acc:.4f} global_samples_per_sec={sums[1].item() / wall:.1f} "
              f"global_tokens_per_sec={sums[2].item() / wall:.1f}", flush=True)
    D.destroy()
    return {"accuracy": acc, "samples": int(sums[1].item()), "seconds": wall}


def test(argv=None):
    p = argparse.ArgumentParser(description="tiny BERT accuracy on test[:512]")
    p.add_argument("--ckpt", default="tiny_out")
    p.add_argument("--batch", type=int, default=32)
    args, _ = p.parse_known_args(argv)
    dev = torch.device("cuda") if torch.cuda.is_available() and os.environ.get("MIFT_DEVICE") != "cpu" \
        else torch.device("cpu")
    model, tok = _load_ckpt(args.ckpt, dev)
    txt, lab, _ = load_split("test", 0, 512)
    data = encode(tok, txt, lab, SEQ)
    corr = 0
    with torch.no_grad():
        for i in range(0, len(lab), args.batch):
            logits = model(input_ids=data["input_ids"][i:i + args.batch].to(dev),
                           attention_mask=data["attention_mask"][i:i + args.batch].to(dev))["logits"]
            corr += int((logits.argmax(-1).cpu() == data["labels"][i:i + args.batch]).sum())
    acc = corr / len(lab)
    print(f"\nAccuracy on 512-row slice: {acc:.3f}")
    print("\n↪ Example predictions")
    for i in random.sample(range(len(lab)), 3):
        with torch.no_grad():
            lg = model(input_ids=data["input_ids"][i:i + 1].to(dev),
                       attention_mask=data["attention_mask"][i:i + 1].to(dev))["logits"]
        print(f"\n• {txt[i][:80]} ...\n  gold={LABELS[lab[i]]:<8}  pred={LABELS[int(lg.argmax(-1))]}")
    return {"accuracy": acc}
