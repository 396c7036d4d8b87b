"""Greedy-generation throughput probe (reference `run_labs45_tiny_final.sbatch:66-89`).

64 identical prompts ("The news today reported that"), ``max_new_tokens=16``,
one warm-up ``generate`` then one timed run; tokens = prompt numel + 64·16;
prints the reference's three lines::

  [RANK 0] INFER global_accuracy=NA
  [RANK 0] INFER global_samples_per_sec=...
  [RANK 0] INFER global_tokens_per_sec=...

plus a JSON line with decode latency.  Weights: random init of the named
architecture unless ``--weights`` points at a local HF checkpoint (no
network); prompt ids are GPT-2 BPE ids of the reference prompt.
"""
import argparse
import json
import time

import torch

from ..infer.generate import generate
from ..models import build_causal_lm

PROMPT_IDS = [464, 1705, 1909, 2098, 326]  # GPT-2 BPE: "The news today reported that"


def distinct_prompts(n, vocab, pad_id, dev, lo=3, hi=12, seed=7):
    """n different prompts of lo..hi tokens, left-padded to the longest -> (ids, mask)."""
    g = torch.Generator().manual_seed(seed)
    lens = [lo + (i * 7) % (hi - lo + 1) for i in range(n)]
    S = max(lens)
    ids = torch.full((n, S), int(pad_id if pad_id is not None and pad_id >= 0 else 0), dtype=torch.long)
    mask = torch.zeros(n, S, dtype=torch.long)
    for i, L in enumerate(lens):
        ids[i, S - L:] = torch.randint(3, vocab, (L,), generator=g)
        mask[i, S - L:] = 1
    return ids.to(dev), mask.to(dev)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="distilgpt2")
    ap.add_argument("--weights", default=None)
    ap.add_argument("--n_prompts", type=int, default=64)
    ap.add_argument("--max_new_tokens", type=int, default=16)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--repeat", type=int, default=1, help="timed generate() calls (best-of)")
    ap.add_argument("--prompts", default="same", choices=["same", "distinct"],
                    help="same: the reference's 64 identical prompts; distinct: 64 different prompts of 3-12 "
                         "tokens, left-padded (tokenizer padding=True, padding_side='left') — the padded path")
    a = ap.parse_args(argv)
    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    if dev.type == "cpu":
        dt = torch.float32
    m = build_causal_lm(a.model, dtype=dt, device=dev, seed=0, weights=a.weights).eval()
    if a.prompts == "same":
        ids = torch.tensor([PROMPT_IDS] * a.n_prompts, device=dev)
        enc_mask = torch.ones_like(ids)
    else:
        ids, enc_mask = distinct_prompts(a.n_prompts, m.config.vocab_size, getattr(m.config, "pad_token_id", 0), dev)
    generate(m, ids, attention_mask=enc_mask, max_new_tokens=a.max_new_tokens, eos_token_id=-1)  # warm-up
    best = float("inf")
    for _ in range(a.repeat):
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = generate(m, ids, attention_mask=enc_mask, max_new_tokens=a.max_new_tokens, eos_token_id=-1)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    tokens = ids.numel() + a.n_prompts * a.max_new_tokens
    print("[RANK 0] INFER global_accuracy=NA")
    print(f"[RANK 0] INFER global_samples_per_sec={a.n_prompts / best:.3f}")
    print(f"[RANK 0] INFER global_tokens_per_sec={tokens / best:.1f}")
    rec = {"model": a.model, "device": str(dev), "dtype": a.dtype, "batch": a.n_prompts, "prompts": a.prompts,
           "prompt_tokens": int(enc_mask.sum()),
           "new_tokens": int(out.shape[1] - ids.shape[1]), "seconds": round(best, 5),
           "ms_per_decode_step": round(best * 1000 / a.max_new_tokens, 3)}
    print(json.dumps(rec), flush=True)
    return rec


if __name__ == "__main__":
    main()
