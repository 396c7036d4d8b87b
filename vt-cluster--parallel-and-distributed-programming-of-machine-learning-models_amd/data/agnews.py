"""AG-News classification data + the BERT WordPiece tokenizer, offline.

Reference (`labs/tiny/train_tiny.py:132-141`, `infer_ddp.py:43-49`,
`test_tiny.py:32-43`): ``load_dataset("ag_news")`` train[:2000]
/ test[:512] (or [:2048]) tokenised to 128 with
``google/bert_uncased_L-2_H-128_A-2``.  No network here, so:

  * the splits are read straight from an HF datasets cache (``ag_news-*.arrow``
    Arrow IPC stream files, via pyarrow — nothing is unpickled) found under
    ``$MIFT_HF_CACHE``, ``$HF_HOME``, ``./.hf_cache`` or
    ``~/.cache/huggingface`` (the product never reads the reference tree; to
    reproduce the reference's own AG-News slice point ``MIFT_HF_CACHE`` at a
    copy of its ``.hf_cache``);
  * when only the test split is cached (as in the reference's own
    ``.hf_cache``, whose train shard is a missing large blob), "train" is
    served from test rows [2048:] — disjoint from every eval slice the labs
    use — and the substitution is reported;
  * with no cache at all, a synthetic 4-class corpus with class-dependent
    vocabulary (learnable, same shapes) stands in.
The WordPiece vocab is located the same way (a cached ``vocab.txt`` blob,
recognised by its ``[PAD]`` / ``[unused0]`` header); fallback: a hashing
word tokenizer with the same special-token ids.
"""
import glob
import os
import re

import numpy as np
import torch

LABELS = ["World", "Sports", "Business", "Sci/Tech"]
TRAIN_FALLBACK_OFFSET = 2048


def cache_roots():
    if os.environ.get("MIFT_AGNEWS") == "synthetic":
        return []
    roots = [os.environ.get("MIFT_HF_CACHE"), os.environ.get("HF_HOME"), os.path.join(os.getcwd(), ".hf_cache"),
             os.path.expanduser("~/.cache/huggingface")]
    return [r for r in roots if r and os.path.isdir(r)]


def _find(pattern):
    for r in cache_roots():
        hits = sorted(glob.glob(os.path.join(r, "**", pattern), recursive=True))
        if hits:
            return hits[0]
    return None


def _read_arrow(path):
    import pyarrow as pa
    with open(path, "rb") as f:
        try:
            t = pa.ipc.open_stream(f).read_all()
        except pa.ArrowInvalid:
            f.seek(0)
            t = pa.ipc.open_file(f).read_all()
    d = t.to_pydict()
    return d["text"], [int(x) for x in d["label"]]


def load_split(split, start=0, stop=None, verbose=True):
    """-> (texts, labels, source) for ``split`` rows [start:stop]."""
    p = _find(f"ag_news-{split}.arrow")
    src = p
    if p is None and split == "train":
        p = _find("ag_news-test.arrow")
        if p is not None:
            start, stop = TRAIN_FALLBACK_OFFSET + start, (TRAIN_FALLBACK_OFFSET + stop) if stop else None
            src = f"{p} [train substitute: rows {TRAIN_FALLBACK_OFFSET}+]"
    if p is None:
        texts, labels = synthetic_agnews(split, (stop or 2048) - start)
        src = "synthetic"
    else:
        texts, labels = _read_arrow(p)
        texts, labels = texts[start:stop], labels[start:stop]
    if verbose:
        print(f"[data] ag_news {split}[{start}:{stop}] <- {src} ({len(texts)} rows)", flush=True)
    return texts, labels, src


def synthetic_agnews(split, n, seed=0):
    rng = np.random.default_rng(seed + (0 if split == "train" else 1))
    topics = [["war", "minister", "election", "treaty", "border", "nation"],
              ["match", "season", "coach", "league", "goal", "team"],
              ["market", "shares", "profit", "bank", "stocks", "oil"],
              ["software", "space", "internet", "research", "computer", "chip"]]
    filler = ["the", "a", "of", "to", "in", "and", "on", "for", "with", "after", "new", "report"]
    texts, labels = [], []
    for _ in range(n):
        y = int(rng.integers(0, 4))
        words = [rng.choice(topics[y]) if rng.random() < 0.35 else rng.choice(filler) for _ in range(24)]
        texts.append(" ".join(words))
        labels.append(y)
    return texts, labels


# ---------------------------------------------------------------- tokenizer
def find_bert_vocab():
    for r in cache_roots():
        for f in glob.glob(os.path.join(r, "**", "*"), recursive=True):
            if os.path.isfile(f) and 100_000 < os.path.getsize(f) < 2_000_000:
                with open(f, "rb") as fh:
                    if fh.read(16).startswith(b"[PAD]\n[unused0]"):
                        return f
    return None


class HashWordTokenizer:
    """Fallback: lower-cased word hashing into a BERT-sized id space ([PAD]=0, [CLS]=101, [SEP]=102)."""
    pad_token_id, cls_token_id, sep_token_id = 0, 101, 102

    def __init__(self, vocab_size=30522):
        self.vocab_size = vocab_size

    def _ids(self, text):
        import zlib
        base = min(1000, self.vocab_size // 2)  # above the special ids; small test vocabs too
        return [base + zlib.crc32(w.encode()) % (self.vocab_size - base) for w in re.findall(r"\w+", text.lower())]

    def __call__(self, texts, max_length=128, **_):
        ids = np.zeros((len(texts), max_length), dtype=np.int64)
        mask = np.zeros_like(ids)
        for i, t in enumerate(texts):
            row = [self.cls_token_id] + self._ids(t)[: max_length - 2] + [self.sep_token_id]
            ids[i, :len(row)] = row
            mask[i, :len(row)] = 1
        return {"input_ids": ids, "attention_mask": mask}

    def save_pretrained(self, d):
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "mift_tokenizer.txt"), "w") as f:
            f.write(f"hashword {self.vocab_size}\n")


def load_bert_tokenizer(path=None):
    """BertTokenizerFast from a checkpoint dir / cached vocab, else HashWordTokenizer."""
    try:
        from transformers import BertTokenizerFast
    except Exception:  # pragma: no cover
        BertTokenizerFast = None
    if path and os.path.isdir(path):
        if os.path.exists(os.path.join(path, "mift_tokenizer.txt")):
            return HashWordTokenizer()
        if BertTokenizerFast and os.path.exists(os.path.join(path, "vocab.txt")):
            return bert_tokenizer_from_vocab(os.path.join(path, "vocab.txt"), BertTokenizerFast)
    vocab = find_bert_vocab()
    if vocab and BertTokenizerFast:
        return bert_tokenizer_from_vocab(vocab, BertTokenizerFast)
    return HashWordTokenizer()


def bert_tokenizer_from_vocab(path, cls=None):
    """WordPiece tokenizer from a vocab.txt-format file (one token per line, id = line number).

    The vocabulary is passed as a token -> id dict: transformers 5 ignores the vocab_file=
    keyword of BertTokenizerFast and silently builds a 5-token (special tokens only) vocabulary,
    which maps every word to [UNK] — the round-3 labs trained on all-[UNK] inputs and sat at chance."""
    if cls is None:
        from transformers import BertTokenizerFast as cls
    with open(path, "r", encoding="utf-8") as f:
        vocab = {ln.rstrip("\n"): i for i, ln in enumerate(f)}
    tok = cls(vocab=vocab, do_lower_case=True)
    if tok.vocab_size != len(vocab):
        raise RuntimeError(f"WordPiece vocabulary from {path}: {tok.vocab_size} of {len(vocab)} tokens loaded")
    return tok


def encode(tok, texts, labels, seq_len=128):
    """-> dict of int64 tensors input_ids/attention_mask [N, seq_len], labels [N]."""
    enc = tok(list(texts), padding="max_length", truncation=True, max_length=seq_len)
    return {"input_ids": torch.as_tensor(np.asarray(enc["input_ids"]), dtype=torch.long),
            "attention_mask": torch.as_tensor(np.asarray(enc["attention_mask"]), dtype=torch.long),
            "labels": torch.as_tensor(labels, dtype=torch.long)}


class TensorBatcher:
    """MicroBatcher protocol over a dict of equal-length tensors (DP-sharded, optional shuffle)."""

    def __init__(self, data, batch, rank=0, world=1, shuffle=True, seed=42, drop_last=False):
        self.data, self.batch, self.rank, self.world = data, batch, rank, world
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.n = len(next(iter(data.values())))
        self.accum = 1

    def indices(self, epoch=0):
        idx = np.arange(self.n)
        if self.shuffle:
            idx = np.random.default_rng(self.seed + epoch).permutation(self.n)
        per = self.n // self.world  # equal shards (DistributedSampler-like, drop the remainder)
        return idx[: per * self.world][self.rank::self.world]

    def steps_per_epoch(self):
        n = len(self.indices(0))
        return n // self.batch if self.drop_last else (n + self.batch - 1) // self.batch

    def epoch(self, epoch=0, start_step=0):
        idx = self.indices(epoch)
        for s in range(start_step, self.steps_per_epoch()):
            j = idx[s * self.batch:(s + 1) * self.batch]
            yield [{k: v[torch.as_tensor(j)] for k, v in self.data.items()}]
