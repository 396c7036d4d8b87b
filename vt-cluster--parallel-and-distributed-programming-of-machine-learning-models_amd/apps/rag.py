"""Retrieval-augmented generation demo: TF-IDF retriever + FLAN-T5 generator.

Reference: `labs/ragging/rag_example.py`.  Same flow and CLI
(``--subset --k --query --queries_file --batch --max_new_tokens --dry_run``):
fit a TF-IDF (1-2 grams, 20k features) retriever over AG-News passages
("train" the retriever), fall back to a token-overlap scorer without
scikit-learn, build the fixed instruction prompt from the top-k passages,
generate with FLAN-T5 (``mift.models.t5``, greedy + KV cache), shard a query
file over ranks (``RANK``/``WORLD_SIZE`` — the reference read LOCAL_RANK
against SLURM_NTASKS).  Offline: the generator is random-init unless
``--weights`` names a local HF checkpoint; the tokenizer is a local HF T5
tokenizer dir (``--tokenizer``) or a SentencePiece unigram model trained on
the retrieval corpus at start-up.
"""
import argparse
import math
import os
import re
import sys
import time
from typing import List, Tuple

import torch

_WS = re.compile(r"\s+")


def norm(txt: str) -> str:
    return _WS.sub(" ", txt.lower()).strip()


def overlap_score(q: str, doc: str) -> float:
    qt, dt = set(norm(q).split()), set(norm(doc).split())
    if not qt or not dt:
        return 0.0
    return len(qt & dt) / math.sqrt(len(qt) * len(dt))


class Retriever:
    """TF-IDF (+ cosine via L2-normalised rows) with a dependency-free overlap fallback."""

    def __init__(self, docs: List[str], force_fallback=False):
        self.docs, self.kind, self.vec, self.mat = docs, "fallback", None, None
        if force_fallback:
            return
        try:
            from sklearn.feature_extraction.text import TfidfVectorizer
            self.vec = TfidfVectorizer(max_features=20_000, ngram_range=(1, 2))
            self.mat = self.vec.fit_transform(docs)
            self.kind = "tfidf"
        except Exception as e:  # pragma: no cover - sklearn is installed here
            print(f"[WARN] scikit-learn unavailable, using overlap fallback: {e}", file=sys.stderr)

    def search(self, query: str, k: int = 3) -> List[Tuple[int, float]]:
        if self.kind == "tfidf":
            import numpy as np
            sims = (self.mat @ self.vec.transform([query]).T).toarray().ravel()
            top = np.argsort(-sims, kind="stable")[:k]
            return [(int(i), float(sims[i])) for i in top]
        scored = sorted(((i, overlap_score(query, d)) for i, d in enumerate(self.docs)), key=lambda x: -x[1])
        return scored[:k]


def build_prompt(query: str, passages: List[str]) -> str:
    ctx = "\n\n".join(f"- {p}" for p in passages)
    return f"Answer the question concisely using the context.\nContext:\n{ctx}\n\nQuestion: {query}\nAnswer:"


class SPTokenizer:
    """SentencePiece unigram tokenizer trained in-process (T5 ids: pad 0, eos 1, unk 2)."""

    def __init__(self, corpus: List[str], vocab_size=4000, model_dir=None):
        import io
        import sentencepiece as spm
        buf = io.BytesIO()
        spm.SentencePieceTrainer.train(sentence_iterator=iter(corpus), model_writer=buf, vocab_size=vocab_size,
                                       model_type="unigram", pad_id=0, eos_id=1, unk_id=2, bos_id=-1,
                                       hard_vocab_limit=False, minloglevel=2)
        self.sp = spm.SentencePieceProcessor(model_proto=buf.getvalue())
        self.vocab_size = self.sp.get_piece_size()

    def __call__(self, text, max_length=512):
        ids = self.sp.encode(text)[: max_length - 1] + [1]
        return {"input_ids": torch.tensor([ids]), "attention_mask": torch.ones(1, len(ids), dtype=torch.long)}

    def decode(self, ids, skip_special_tokens=True):
        ids = [int(i) for i in ids if not (skip_special_tokens and int(i) in (0, 1))]
        return self.sp.decode(ids)


class HFTokenizerAdapter:
    def __init__(self, path):
        from transformers import AutoTokenizer
        self.tok = AutoTokenizer.from_pretrained(path)
        self.vocab_size = len(self.tok)

    def __call__(self, text, max_length=512):
        return self.tok(text, return_tensors="pt", truncation=True, max_length=max_length)

    def decode(self, ids, skip_special_tokens=True):
        return self.tok.decode(ids, skip_special_tokens=skip_special_tokens)


def build_generator(args, tok, device):
    from ..models import load_hf_weights
    from ..models.t5 import T5Config, T5ForConditionalGeneration
    cfg = T5Config.preset(args.generator)
    if args.weights is None:
        cfg.vocab_size = max(cfg.vocab_size if args.tokenizer else 0, tok.vocab_size)
    gen = T5ForConditionalGeneration(cfg, device=device)
    if args.weights:
        load_hf_weights(gen, args.weights)
    else:
        gen.init_weights(0)
    return gen.eval()


def main(argv=None):
    ap = argparse.ArgumentParser(description="RAG demo: TF-IDF retriever + FLAN-T5 generator")
    ap.add_argument("--subset", type=int, default=2000)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--query", default=None)
    ap.add_argument("--queries_file", default=None)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--max_new_tokens", type=int, default=64)
    ap.add_argument("--dry_run", action="store_true")
    ap.add_argument("--generator", default="flan-t5-small")
    ap.add_argument("--weights", default=None, help="local HF checkpoint dir of the generator")
    ap.add_argument("--tokenizer", default=None, help="local HF T5 tokenizer dir")
    ap.add_argument("--fallback_retriever", action="store_true")
    ap.add_argument("--show_passages", action="store_true", help="also print the retrieved passages (score, text)")
    args, _ = ap.parse_known_args(argv)
    from ..data.agnews import load_split
    n = min(args.subset, 2000) if args.dry_run else args.subset
    texts, _, src = load_split("train", 0, n)
    corpus = [t.strip(" -") for t in texts]
    t0 = time.time()
    retr = Retriever(corpus, force_fallback=args.fallback_retriever)
    print(f"[retriever] kind={retr.kind} trained_on={len(corpus)} docs in {time.time() - t0:.2f}s", flush=True)
    tok = HFTokenizerAdapter(args.tokenizer) if args.tokenizer else SPTokenizer(corpus)
    dev = torch.device("cuda") if torch.cuda.is_available() and os.environ.get("MIFT_DEVICE") != "cpu" \
        else torch.device("cpu")
    gen = build_generator(args, tok, dev)

    def answer(q):
        hits = retr.search(q, k=args.k)
        enc = tok(build_prompt(q, [corpus[i] for i, _ in hits]))
        out = gen.generate(enc["input_ids"].to(dev), enc["attention_mask"].to(dev), max_new_tokens=args.max_new_tokens)
        return tok.decode(out[0].tolist()), hits

    results = []
    if args.query:
        a, hits = answer(args.query)
        print("\nQ:", args.query)
        print("A:", a)
        return [(args.query, a, hits)]
    if args.queries_file and os.path.exists(args.queries_file):
        with open(args.queries_file, encoding="utf-8") as fh:
            queries = [ln.strip() for ln in fh if ln.strip()]
        rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
        shard = queries[rank::world]
        print(f"[rank {rank}/{world}] processing {len(shard)} queries", flush=True)
        for i in range(0, len(shard), args.batch):
            for q in shard[i:i + args.batch]:
                a, hits = answer(q)
                print(f"\nQ: {q}\nA: {a}", flush=True)
                if args.show_passages:
                    for i, sc in hits:
                        print(f"   [{sc:.3f}] {corpus[i][:110]}", flush=True)
                results.append((q, a, hits))
        return results
    print("Nothing to do: provide --query '...' or --queries_file <path>.")
    return results
