"""Data: text-line datasets, pre-tokenized dirs, synthetic OpenWebText-shaped
token streams, LM collation and DP-rank sharding.

Reference behaviour:
  * ``load_dataset("text", data_files=...)`` — one example per line, empty
    lines kept (``P1/finetune_lora_distilgpt2.py:67-71``);
  * tokenize with truncation + ``padding="max_length"``, right padding, pad =
    eos (``P1/...:84-86,107-108``);
  * ``DataCollatorForLanguageModeling(mlm=False)``: labels = input_ids with
    pad positions set to -100 (pad == eos, so real EOS tokens are masked
    too — B17, kept for parity);
  * pre-tokenized ``save_to_disk`` dirs with input_ids/attention_mask
    (``P2/finetune_lora_opt_pp.py:61-89``);
  * sharding: Trainer DistributedSampler (strided) for DDP, contiguous for
    P2 — by DP rank, not global rank (fixes B7).

Everything is materialised as one int32 token matrix [N, S] + lengths, so a
micro-batch is a row slice (pinned host memory -> async H2D).
"""
import os

import numpy as np
import torch


class TokenDataset:
    """N fixed-length examples: ids [N, S] int32, lengths [N] int32."""

    def __init__(self, ids: np.ndarray, lengths: np.ndarray, pad_id: int, vocab_size: int):
        assert ids.ndim == 2
        self.ids = np.ascontiguousarray(ids, dtype=np.int32)
        self.lengths = np.ascontiguousarray(lengths, dtype=np.int32)
        self.pad_id, self.vocab_size = pad_id, vocab_size

    def __len__(self):
        return self.ids.shape[0]

    @property
    def seq_len(self):
        return self.ids.shape[1]

    def batch(self, idx):
        """-> dict(input_ids int64 [b,S], attention_mask int64, labels int64) (CPU)."""
        ids = torch.from_numpy(self.ids[idx].astype(np.int64))
        lens = torch.from_numpy(self.lengths[idx].astype(np.int64))
        S = ids.shape[1]
        mask = (torch.arange(S)[None, :] < lens[:, None]).long()
        return {"input_ids": ids, "attention_mask": mask, "labels": lm_labels(ids, mask, self.pad_id)}

    def save(self, path):
        os.makedirs(path, exist_ok=True)
        np.save(os.path.join(path, "ids.npy"), self.ids)
        np.save(os.path.join(path, "lengths.npy"), self.lengths)
        with open(os.path.join(path, "meta.txt"), "w") as f:
            f.write(f"{self.pad_id} {self.vocab_size}\n")

    @staticmethod
    def load(path):
        ids = np.load(os.path.join(path, "ids.npy"), allow_pickle=False)
        lens = np.load(os.path.join(path, "lengths.npy"), allow_pickle=False)
        with open(os.path.join(path, "meta.txt")) as f:
            pad, vocab = map(int, f.read().split())
        return TokenDataset(ids, lens, pad, vocab)


def row_label_tokens(ds: "TokenDataset") -> np.ndarray:
    """[N] int64: per-row count of shifted causal-LM targets (labels[1:] != -100, see lm_labels)."""
    cached = getattr(ds, "_row_label_tokens", None)
    if cached is not None:
        return cached
    S = ds.ids.shape[1]
    out = np.empty(len(ds), dtype=np.int64)
    cols = np.arange(1, S)[None, :]
    for r0 in range(0, len(ds), 16384):  # bounded temporaries on large corpora
        ids = ds.ids[r0:r0 + 16384, 1:]
        lens = ds.lengths[r0:r0 + 16384, None]
        out[r0:r0 + len(ids)] = ((cols < lens) & (ids != ds.pad_id)).sum(axis=1)
    ds._row_label_tokens = out
    return out


class StepBatch(list):
    """The micro-batches of one optimizer step; ``global_tokens`` = label tokens over all DP ranks."""
    global_tokens = None


def lm_labels(ids: torch.Tensor, mask: torch.Tensor, pad_id: int) -> torch.Tensor:
    """Causal-LM labels: input_ids with padding (and pad-id tokens) -> -100."""
    lab = ids.clone()
    lab[mask == 0] = -100
    lab[ids == pad_id] = -100
    return lab


def synthetic_openwebtext(n_lines: int, seq_len: int, vocab_size: int, pad_id: int, seed: int = 0,
                          full_length: bool = True, mean_tokens: int = 220) -> TokenDataset:
    """Random token lines shaped like the reference's OpenWebText line files.

    ``full_length=True`` (bench default): every line fills ``seq_len`` —
    padded-token throughput equals real-token throughput.  Otherwise line
    lengths ~ clipped geometric around ``mean_tokens`` and right padding."""
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, vocab_size - 1, size=(n_lines, seq_len), dtype=np.int64)
    ids[ids == pad_id] = (pad_id + 1) % (vocab_size - 1)
    if full_length:
        lens = np.full(n_lines, seq_len, dtype=np.int32)
    else:
        lens = np.clip(rng.geometric(1.0 / mean_tokens, size=n_lines), 1, seq_len).astype(np.int32)
        cols = np.arange(seq_len)[None, :]
        ids = np.where(cols < lens[:, None], ids, pad_id)
    return TokenDataset(ids.astype(np.int32), lens, pad_id, vocab_size)


def read_text_lines(path: str):
    """HF ``load_dataset('text')`` semantics: one example per line (newline stripped)."""
    with open(path, "r", encoding="utf-8", errors="replace") as f:
        return [ln.rstrip("\n").rstrip("\r") for ln in f]


def tokenize_lines(lines, tokenizer, seq_len: int, pad_id: int, vocab_size: int) -> TokenDataset:
    """Truncate + right-pad to ``seq_len`` (``padding='max_length'``)."""
    n = len(lines)
    ids = np.full((n, seq_len), pad_id, dtype=np.int32)
    lens = np.zeros(n, dtype=np.int32)
    enc = tokenizer.encode_batch(lines)
    for i, e in enumerate(enc):
        t = e[:seq_len]
        ids[i, : len(t)] = t
        lens[i] = len(t)
    return TokenDataset(ids, lens, pad_id, vocab_size)


def is_saved_dataset_dir(p: str) -> bool:
    """P2 ``_is_saved_dataset_dir``: HF save_to_disk dir or our npy token dir."""
    return os.path.isdir(p) and (os.path.exists(os.path.join(p, "dataset_info.json"))
                                 or os.path.exists(os.path.join(p, "ids.npy")))


def load_pretokenized(path: str, seq_len: int, pad_id: int, vocab_size: int) -> TokenDataset:
    if os.path.exists(os.path.join(path, "ids.npy")):
        return TokenDataset.load(path)
    # HF datasets save_to_disk dir with input_ids / attention_mask columns (arrow)
    from datasets import load_from_disk
    ds = load_from_disk(path)
    if hasattr(ds, "keys") and "train" in ds:
        ds = ds["train"]
    ids = np.full((len(ds), seq_len), pad_id, dtype=np.int32)
    lens = np.zeros(len(ds), dtype=np.int32)
    for i, row in enumerate(ds):
        t = list(row["input_ids"])[:seq_len]
        m = list(row.get("attention_mask", [1] * len(t)))[:seq_len]
        ids[i, : len(t)] = t
        lens[i] = int(sum(m))
    return TokenDataset(ids, lens, pad_id, vocab_size)


def shard_indices(n: int, rank: int, world: int, mode: str = "strided", shuffle: bool = False,
                  seed: int = 0, epoch: int = 0, drop_last: bool = False) -> np.ndarray:
    """DistributedSampler-like sharding by (DP) rank.

    ``strided``: torch DistributedSampler (pad by wrapping so every rank gets
    ceil(n/world) samples); ``contiguous``: HF ``Dataset.shard(contiguous=True)``."""
    order = np.arange(n)
    if shuffle:
        order = np.random.default_rng(seed + epoch).permutation(n)
    if mode == "contiguous":
        div, mod = divmod(n, world)
        start = rank * div + min(rank, mod)
        end = start + div + (1 if rank < mod else 0)
        return order[start:end]
    per = (n + world - 1) // world if not drop_last else n // world
    total = per * world
    if total > n:
        order = np.concatenate([order, order[: total - n]])
    else:
        order = order[:total]
    return order[rank:total:world]


class MicroBatcher:
    """Yields optimizer steps as lists of `accum` micro-batches for one rank.

    Host tensors are pinned so the H2D copy is asynchronous (non_blocking).  With the extension
    available the batches come from the native prefetching loader (csrc/runtime/loader.cpp:
    a C++ worker thread gathers rows, builds masks / labels into pinned tensors ahead of the
    consumer); ``native=False`` or ``MIFT_NATIVE_LOADER=0`` selects the Python path (same
    batches, element for element)."""

    def __init__(self, ds: TokenDataset, micro_batch: int, accum: int, rank: int = 0, world: int = 1,
                 mode: str = "strided", shuffle: bool = False, seed: int = 0, pin: bool = True,
                 native=None, prefetch: int = 4):
        self.ds, self.mb, self.accum = ds, micro_batch, accum
        self.rank, self.world, self.mode, self.shuffle, self.seed = rank, world, mode, shuffle, seed
        self.pin = pin and torch.cuda.is_available()
        if native is None:
            native = os.environ.get("MIFT_NATIVE_LOADER", "1") != "0"
        self.native = bool(native) and _native_loader_available()
        self.prefetch = prefetch
        self._loader = None

    def indices(self, epoch=0, rank=None):
        r = self.rank if rank is None else rank
        return shard_indices(len(self.ds), r, self.world, self.mode, self.shuffle, self.seed, epoch)

    def global_step_tokens(self, epoch=0):
        """[steps] int64: shifted causal-LM label tokens of each optimizer step summed over ALL DP ranks.

        The shard plan is deterministic, so every rank computes the same counts locally: the
        token-normalised loss needs no per-step collective (the reference Trainer all-gathers
        ``num_items_in_batch`` every step)."""
        key = (epoch,)
        if getattr(self, "_gst", (None,))[0] == key:
            return self._gst[1]
        rows = row_label_tokens(self.ds)
        per = self.mb * self.accum
        tot = None
        for r in range(self.world):
            idx = self.indices(epoch, rank=r)
            c = rows[idx]
            starts = np.arange(0, len(c), per)
            s = np.add.reduceat(c, starts) if len(c) else np.zeros(0, np.int64)
            if tot is None:
                tot = s
            else:  # contiguous shards may differ by a step between ranks: zero-pad the shorter
                n = max(len(tot), len(s))
                tot = np.pad(tot, (0, n - len(tot))) + np.pad(s, (0, n - len(s)))
        self._gst = (key, tot.astype(np.int64))
        return self._gst[1]

    def steps_per_epoch(self):
        n = len(self.indices(0))
        return (n + self.mb * self.accum - 1) // (self.mb * self.accum)

    def sample_step(self):
        """One full-shape optimizer step (``accum`` micro-batches of ``mb`` rows) built from the first
        rows of the dataset, without touching the epoch iterators — the Trainer's setup-time warm-up
        and graph capture use its shapes; its values never reach the model's parameters."""
        n = min(self.mb, len(self.ds))
        b = self.ds.batch(np.arange(n))
        if n < self.mb:  # tiny datasets: repeat rows to the full micro-batch shape
            rep = (self.mb + n - 1) // n
            b = {k: v.repeat(rep, 1)[:self.mb] for k, v in b.items()}
        step = StepBatch(dict(b) for _ in range(self.accum))
        step.global_tokens = None
        return step

    def micro_batches_per_epoch(self):
        n = len(self.indices(0))
        return (n + self.mb - 1) // self.mb

    def _native_epoch(self, idx, start_step):
        from .. import _ext
        if self._loader is None:
            self._loader = _ext.require().TokenLoader(torch.from_numpy(self.ds.ids), torch.from_numpy(self.ds.lengths),
                                                      int(self.ds.pad_id), int(self.mb), int(self.prefetch),
                                                      bool(self.pin))
        n_mb = (len(idx) + self.mb - 1) // self.mb
        first = start_step * self.accum
        self._loader.start(torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64)), first)
        step_mbs, j = StepBatch(), first
        while True:
            item = self._loader.next()
            if not item:
                break
            step_mbs.append({"input_ids": item[0], "attention_mask": item[1], "labels": item[2]})
            j += 1
            if len(step_mbs) == self.accum or j == n_mb:
                yield step_mbs
                step_mbs = StepBatch()

    def epoch(self, epoch=0, start_step=0):
        idx = self.indices(epoch)
        gtok = self.global_step_tokens(epoch)
        it = self._native_epoch(idx, start_step) if self.native else self._py_epoch(idx, start_step)
        for s, step_mbs in enumerate(it, start=start_step):
            step_mbs.global_tokens = int(gtok[s]) if s < len(gtok) else None
            yield step_mbs

    def _py_epoch(self, idx, start_step):
        n_mb = (len(idx) + self.mb - 1) // self.mb
        step_mbs = StepBatch()
        for j in range(n_mb):
            b = self.ds.batch(idx[j * self.mb:(j + 1) * self.mb])
            if self.pin:
                b = {k: v.pin_memory() for k, v in b.items()}
            step_mbs.append(b)
            if len(step_mbs) == self.accum or j == n_mb - 1:
                step_no = j // self.accum
                if step_no >= start_step:
                    yield step_mbs
                step_mbs = StepBatch()


def _native_loader_available():
    try:
        from .. import _ext
        return _ext.available() and hasattr(_ext.require(), "TokenLoader")
    except Exception:
        return False
