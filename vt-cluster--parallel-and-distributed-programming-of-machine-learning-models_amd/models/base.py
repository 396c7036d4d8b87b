"""Shared machinery of the causal-LM families (GPT-2, OPT).

Every family exposes the same engine-facing surface so the DDP trainer,
the pipeline engine and the generator treat them alike:

  * ``forward(input_ids, attention_mask, labels, hidden_states, ...)`` ->
    ``{"loss", "logits", "ntokens"}`` on the head stage, ``{"hidden_states"}``
    on a stage without a head (``layer_range`` / ``has_embed`` / ``has_head``
    build only one pipeline stage's weights: SURVEY §6 — the reference OOMs
    because every rank materialises the whole fp32 model first);
  * interleaved pipeline stages (``parallel/pipeline.py``, virtual stages): ``layer_range`` may
    be a LIST of (lo, hi) chunks (OPT: bounds on half layers, ``normalize_chunks``); the pipeline engine selects one with ``active_chunk`` before a
    forward, which then runs only that chunk's blocks, the embedding only on the first chunk of the
    first stage and the head only on the last chunk of the last stage;
  * ``seed`` / ``micro_step``: counter-based dropout seeds, so a block
    recomputed under activation checkpointing — or re-run by the pipeline
    engine's backward — draws bit-identical masks;
  * ``lm_weight_padded()``: the tied LM head as a [V_pad, d] operand
    (V rounded up to 128 so the GEMM and the xent kernel see aligned rows).
"""
import torch
import torch.nn as nn

from ..ops.dispatch import use_kernels
from .layers import dropout_seed, seed_for


def _on_grid(x, step):
    return abs(x / step - round(x / step)) < 1e-9


def normalize_chunks(layer_range, n_layers, halves=False):
    """``layer_range``: None (all layers), (lo, hi), or [(lo, hi), ...] (interleaved chunks)
    -> (span (lo, hi), chunk list, per-layer membership).  ``halves`` (OPT): bounds may fall on half
    layers — unit 2i is layer i's attention sub-block (LN, q/k/v, attention, out_proj + residual),
    unit 2i + 1 its MLP sub-block — so a pipeline boundary can split a decoder layer at its residual
    stream (``chunk_parts``)."""
    if layer_range is None:
        chunks = [(0, n_layers)]
    elif isinstance(layer_range[0], (tuple, list)):
        chunks = [tuple(c) for c in layer_range]
    else:
        chunks = [tuple(layer_range)]
    step = 0.5 if halves else 1
    for lo, hi in chunks:
        if not (0 <= lo < hi <= n_layers) or not (_on_grid(lo, step) and _on_grid(hi, step)):
            raise ValueError(f"bad layer chunk {(lo, hi)} for {n_layers} layers"
                             + ("" if halves else " (whole layers only for this model)"))
    member = [any(lo < i + 1 and i < hi for lo, hi in chunks) for i in range(n_layers)]
    return (min(c[0] for c in chunks), max(c[1] for c in chunks)), chunks, member


def chunk_parts(chunks, i):
    """(attention sub-block, MLP sub-block) of layer ``i`` inside any of ``chunks``."""
    return (any(lo <= i and i + 0.5 <= hi for lo, hi in chunks),
            any(lo <= i + 0.5 and i + 1 <= hi for lo, hi in chunks))


class CausalLMBase(nn.Module):
    active_chunk = None  # interleaved pipeline: index into chunk_ranges run by forward (None: all)

    def blocks(self):
        """The decoder blocks this module runs: all of its blocks, or those of ``active_chunk``."""
        bl = self.all_blocks()
        if self.active_chunk is None:
            return bl
        lo, hi = self.chunk_ranges[self.active_chunk]
        return [b for b in bl if lo < b.idx + 1 and b.idx < hi]

    def block_parts(self, blk):
        """(attention, MLP) sub-blocks of ``blk`` this forward runs (half-layer pipeline chunks)."""
        chunks = self.chunk_ranges if self.active_chunk is None else [self.chunk_ranges[self.active_chunk]]
        return chunk_parts(chunks, blk.idx)

    @property
    def embed_here(self):
        return self.has_embed and self.active_chunk in (None, 0)

    @property
    def head_here(self):
        return self.has_head and self.active_chunk in (None, len(self.chunk_ranges) - 1)

    def _init_runtime(self, vocab_padded):
        self.vocab_padded = vocab_padded
        self.seed = 0
        self.micro_step = 0
        self.fused = True  # use HIP kernels for GPU tensors
        self.recompute = False
        self._head_cache = None

    # subclasses: tied_embedding() -> nn.Parameter [V, d]; blocks() -> list

    def lm_weight_padded(self, transposed=False):
        """Tied LM head as ([V_pad, d], [d, V_pad] or None) with zero rows beyond the vocab.

        The [d, V_pad] copy (K-contiguous B operand of the fused head's dgrad, ops/fused.py) is
        built on first request and cached with the padded weight (frozen: built once)."""
        w = self.tied_embedding()
        key = (w.data_ptr(), w.dtype, w.device)
        if self._head_cache is None or self._head_cache[0] != key:
            wp = torch.zeros(self.vocab_padded, w.shape[1], dtype=w.dtype, device=w.device)
            wp[: w.shape[0]].copy_(w.detach())
            self._head_cache = (key, wp, None)
        if transposed and self._head_cache[2] is None:
            self._head_cache = (key, self._head_cache[1], self._head_cache[1].t().contiguous())
        return self._head_cache[1], self._head_cache[2]

    def next_micro_step(self):
        self.micro_step += 1

    def embed_seed(self):
        return dropout_seed(self.seed, self.micro_step, 1)

    def _use_fused(self, t):
        return self.fused and use_kernels(t)

    def num_layers(self):
        return self.config.num_layers()

    # ---- generation hooks (mift.infer.generate) ----
    POS_OFFSET = 0

    def embed_at(self, ids, pos):
        """Token + learned-position embedding for explicit positions (no dropout)."""
        wte, wpe = self.embedding_tables()
        if self._use_fused(ids):
            from ..ops import kernels as K
            B, S = ids.shape
            return K.embed(ids.contiguous(), wte.weight, wpe.weight, pos=pos.contiguous(),
                           pos_offset=self.POS_OFFSET).view(B, S, -1)
        return wte(ids) + wpe(pos + self.POS_OFFSET)

    def head_logits(self, h):
        """[B, S, d] -> [B, S, V] through the final LayerNorm and the tied head."""
        if self._use_fused(h):
            from ..ops import fused as F
            return F.lm_head_logits(h, self.final_norm(), self.lm_weight_padded()[0], self.config.vocab_size)
        return self.final_norm()(h) @ self.tied_embedding().t()

    def stage_parameters(self):
        """(name, tensor) of everything this stage materialised (for memory reports)."""
        return list(self.named_parameters())


def shift_labels(labels, ignore_index=-100):
    """labels[:, 1:] with an ignore column appended -> aligned with every row."""
    out = torch.full_like(labels, ignore_index)
    out[:, :-1] = labels[:, 1:]
    return out


def ref_lm_loss(logits, labels, ignore_index=-100, reduction="mean"):
    """HF shifted causal-LM CE (fp32 logits)."""
    sl = logits[:, :-1].reshape(-1, logits.shape[-1])
    tl = labels[:, 1:].reshape(-1)
    return torch.nn.functional.cross_entropy(sl.float(), tl, ignore_index=ignore_index, reduction=reduction)
