"""Greedy generation with a KV cache (K12) for the causal-LM families.

Reference: HF ``model.generate(**enc, max_new_tokens=16)`` on distilgpt2 in
the lab generation probe (`run_labs45_tiny_final.sbatch:66-89`, SURVEY
§3.5 / C42) and FLAN-T5 generation in the RAG lab.  Semantics kept from HF
greedy search: left-padded batches, positions from the attention mask
(GPT-2: cumsum(mask)-1; OPT: the same + offset 2), a finished row keeps
emitting ``pad_token_id`` after ``eos_token_id``, stop when every row is
finished.

MI355X design: one preallocated cache per layer ``[B, H, Tmax, hd]`` (16-bit,
HBM-resident — 288 GB makes Tmax = context limit affordable), prefill runs
the normal block path through the flash-attention kernel and stores K/V once;
every decode step is the fused block path with the attention replaced by
the ``decode_attn`` HIP kernel, which appends the new K/V in the same
launch, and the LM-head logits are the hand-written MFMA GEMM (``gemm_nt``).
No library GEMM and no SDPA run on the GPU path.

A whole call — prefill, token 0 and every decode step — is replayed from ONE hipGraph
(``_DecodeGraph``; ``MIFT_GEN_GRAPH=0`` disables): a step is ~34 kernels of a few microseconds each, so
eagerly it was host-launch bound (0.62 ms per step for distilgpt2 at batch 64),
and the eager prefill spent 1.67 ms of span on 0.61 ms of kernels (round 5).  Everything a step
varies lives on the device — the cache position (``decode_attn`` reads it from an int32 tensor), the
positions, the finished-row flags and the output column — and advances inside the graph, so the
steps are identical captures and, cached per (model, batch, prompt length, budget), one graph serves
every later call of the same shape (its ids and prompt lengths are copied into static inputs).  HF's
stop-when-all-finished rule is applied afterwards: the steps past the last row's EOS only produce
pad tokens and are trimmed (no per-step host sync).

Left-padded batches: the prefill runs every prompt RIGHT-aligned to position 0
(row b's tokens ``ids[b, start_b:]`` then padding) so the flash kernel's
``kv_len`` key mask is exact — queries see keys [0, q] of their own prompt,
positions are 0..len_b-1 as HF computes them from the mask — and the next
token is read at row b's last prompt position.  The cache then holds row b's
prompt at [0, len_b) and generated tokens from S0 on; the decode kernel masks
the gap [len_b, S0).  Returned ids keep the HF left-padded layout.  CPU
tensors run the same algorithm with torch ops (the oracle).
"""
import gc
import os
import weakref

import numpy as np
import torch

from ..ops import reference as ref


class KVCache:
    def __init__(self, n_layers, B, H, Tmax, hd, dtype, device):
        shape = (B, H, Tmax, hd)
        self.k = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(n_layers)]
        self.v = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(n_layers)]
        self.Tmax = Tmax

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in self.k + self.v)


def _split_heads(x, B, S, H, hd):
    return x.view(B, S, H, hd).transpose(1, 2)


def _prefill_attn(cache, li, B, S, H, hd, kv_len, fused):
    """attn(qkv [B,S,3d]) -> o [B,S,d] over right-aligned prompts (keys >= kv_len[b] masked);
    stores K/V rows [0, S) of layer li."""
    d = H * hd
    scale = hd ** -0.5

    def attn(qkv):
        qkv3 = qkv.reshape(B, S, 3 * d)
        if fused:
            from ..ops import kernels as K
            from ..ops.attention import causal_attention
            K.kv_store(qkv.reshape(B * S, 3 * d).contiguous(), cache.k[li], cache.v[li], S)
            return causal_attention(qkv3, B, S, H, hd, scale=scale, kv_len=kv_len)
        k = _split_heads(qkv3[..., d:2 * d], B, S, H, hd)
        v = _split_heads(qkv3[..., 2 * d:], B, S, H, hd)
        cache.k[li][:, :, :S].copy_(k)
        cache.v[li][:, :, :S].copy_(v)
        q = _split_heads(qkv3[..., :d], B, S, H, hd)
        valid = None
        if kv_len is not None:
            valid = torch.arange(S, device=qkv.device)[None, :] < kv_len[:, None].long()
        o = ref.attention(q, k, v, causal=True, key_padding=valid, scale=scale)
        return o.transpose(1, 2).reshape(B, S, d)

    return attn


def _decode_attn(cache, li, B, H, hd, t, plen, gend, fused):
    """Attention of the token at cache position t; keys in [plen[b], gend) are the prompt gap."""
    d = H * hd
    scale = hd ** -0.5

    def attn(qkv):
        if fused:
            from ..ops import kernels as K
            o = K.decode_attn(qkv.reshape(B, 3 * d).contiguous(), cache.k[li], cache.v[li], t, scale,
                              plen=plen, gend=gend)
            return o.view(B, 1, d)
        qkv3 = qkv.reshape(B, 3 * d)
        q = qkv3[:, :d].view(B, H, 1, hd)
        cache.k[li][:, :, t] = qkv3[:, d:2 * d].view(B, H, hd)
        cache.v[li][:, :, t] = qkv3[:, 2 * d:].view(B, H, hd)
        k, v = cache.k[li][:, :, :t + 1], cache.v[li][:, :, :t + 1]
        valid = None
        if plen is not None:
            j = torch.arange(t + 1, device=qkv.device)[None, :]
            valid = (j < plen[:, None].long()) | (j >= gend)
        o = ref.attention(q, k, v, causal=False, key_padding=valid, scale=scale)
        return o.transpose(1, 2).reshape(B, 1, d)

    return attn


def _run_blocks(model, h, attn_for_layer, fused):
    for li, blk in enumerate(model.blocks()):
        s = blk.site_seeds(0, 0)  # eval: no dropout is drawn
        if fused:
            h = blk.forward_fused(h, s, False, attn=attn_for_layer(li))
        else:
            h = blk.forward_ref(h, s, False, attn=attn_for_layer(li))
    return h


def _heads(model):
    blk = model.blocks()[0]
    a = getattr(blk, "attn", None) or getattr(blk, "self_attn")
    return a.n_head, a.head_dim


class _DecodeGraph:
    """One greedy generate() call of a fixed shape over static device state: the prefill, token 0's
    argmax / bookkeeping and every decode step, captured as ONE hipGraph (see the module docstring).

    The first call of a shape runs the same sequence eagerly (its result is that call's output) and
    then captures it; later calls copy their ids / prompt lengths into the static inputs and replay
    once.  The prefill was ~90 host-issued kernels with 10-20 us of launch gap each (1.67 ms span for
    0.61 ms of kernels at batch 64, ``profiles/r5/gen_timeline_r5k.txt``) and every decode step one
    replay of its own."""

    def __init__(self, model, B, S0, max_new, padded, pad, eos, fill, H, hd, dtype, dev):
        self.key = (B, S0, max_new, padded, pad, eos, fill)
        # the graph holds raw pointers to the model's weights; the cache holds the model only weakly
        # (a dead or different model under the same id() evicts the entry in _decode_graph)
        self.model_ref = weakref.ref(model)
        L = len(model.blocks())
        self.cache = KVCache(L, B, H, S0 + max_new, hd, dtype, dev)
        self.B, self.S0, self.H, self.hd, self.fill, self.pad, self.eos = B, S0, H, hd, fill, pad, eos
        self.max_new, self.padded = max_new, padded
        self.in_ids = torch.zeros(B, S0, dtype=torch.long, device=dev)  # static inputs of a call
        self.in_lens = torch.zeros(B, dtype=torch.long, device=dev)
        self.lens_pin = torch.zeros(B, dtype=torch.long, pin_memory=True)  # host side of in_lens' upload
        self.lens_ev = None
        self.ids = torch.zeros(B, 1, dtype=torch.long, device=dev)  # this step's input token per row
        self.done = torch.zeros(B, dtype=torch.bool, device=dev)
        self.t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.pos = torch.zeros(B, 1, dtype=torch.long, device=dev)
        self.col = torch.zeros(B, 1, dtype=torch.long, device=dev)
        self.out = torch.zeros(B, max_new, dtype=torch.long, device=dev)
        self.plen = torch.zeros(B, dtype=torch.int32, device=dev) if padded else None
        self.graph = self.step_graph = None

    def prefill(self, model):
        """Prompts (static in_ids / in_lens) through the model, K/V rows [0, S0) of every layer cached,
        then token 0: argmax of each row's last prompt position through ``decode_tail`` with the state
        set so that it leaves t = S0, pos = len, col = 1 (HF: a row is finished once it emits EOS)."""
        from ..ops import kernels as K
        B, S0, H, hd = self.B, self.S0, self.H, self.hd
        dev = self.in_ids.device
        ar = torch.arange(S0, device=dev)
        lens = self.in_lens
        if self.padded:  # right-align every prompt to position 0 (see generate)
            self.plen.copy_(lens)
            src = (ar[None, :] + (S0 - lens)[:, None]).clamp(max=S0 - 1)
            ids_r = torch.where(ar[None, :] < lens[:, None], torch.gather(self.in_ids, 1, src),
                                torch.full_like(self.in_ids, self.fill))
        else:
            ids_r = self.in_ids
        h = model.embed_at(ids_r, ar[None, :].expand(B, S0).contiguous())
        h = _run_blocks(model, h, lambda li: _prefill_attn(self.cache, li, B, S0, H, hd, self.plen, True), True)
        if self.padded:
            last = (lens - 1).clamp(min=0)
            h_last = torch.gather(h, 1, last[:, None, None].expand(B, 1, h.shape[-1]))
        else:
            h_last = h[:, -1:]
        logits = model.head_logits(h_last)[:, -1]
        self.done.zero_()
        self.col.zero_()
        self.out.zero_()
        self.t.fill_(S0 - 1)
        self.pos.copy_((lens - 1)[:, None])
        K.decode_tail(logits, logits.shape[-1], self.done, self.ids, self.out, self.col, self.pos, self.t, self.fill,
                      self.pad, self.eos)

    def step(self, model):
        """One decode step on the static state.  The greedy tail — argmax, pad for finished rows, the
        output column, EOS flags, the next input ids and the position / column / cache-position
        advance — is ONE kernel (``decode_tail``; it was ~12 torch kernels per step)."""
        from ..ops import kernels as K
        B, H, hd = self.B, self.H, self.hd
        h = model.embed_at(self.ids, self.pos)
        h = _run_blocks(model, h, lambda li: _decode_attn(self.cache, li, B, H, hd, self.t, self.plen, self.S0, True),
                        True)
        logits = model.head_logits(h)[:, -1]
        K.decode_tail(logits, logits.shape[-1], self.done, self.ids, self.out, self.col, self.pos, self.t, self.fill,
                      self.pad, self.eos)

    def call(self, model):
        self.prefill(model)
        for _ in range(self.max_new - 1):
            self.step(model)

    def run(self, model, input_ids, lens):
        """Tokens [B, max_new] of one call (static output; the caller copies it out).  ``lens``: host
        int64 prompt lengths (uploaded through a pinned buffer)."""
        self.in_ids.copy_(input_ids)
        if self.lens_ev is not None:
            self.lens_ev.synchronize()  # the previous call's upload has read the pinned buffer
        self.lens_pin.copy_(lens)
        self.in_lens.copy_(self.lens_pin, non_blocking=True)
        self.lens_ev = torch.cuda.Event()
        self.lens_ev.record()
        if self.graph is not None:
            self._replay()
            return self.out
        self.call(model)  # first call of this shape: eager (first launch of every kernel module) ...
        # ... then the capture, which must rebuild every cached LoRA operand pack INSIDE the graph (each
        # replay then re-packs from the live adapter weights); without this the eager pass's packs, built
        # at the same arena version, are baked in and a later call that replaces them leaves the replays
        # reading freed memory.  The eager pass's tokens are kept aside: the capture itself
        # runs nothing, but it must not race the copy-out.
        toks = self.out.clone()
        from ..ops.fused import invalidate_packs
        invalidate_packs(model)
        # up to MIFT_GEN_UNROLL (64) steps are unrolled into the one graph; longer budgets capture the
        # prefill and ONE step and replay the step graph per token (graph size stays ~35 nodes per step)
        unroll = self.max_new - 1 <= int(os.environ.get("MIFT_GEN_UNROLL", "64"))
        was = gc.isenabled()
        gc.collect()
        gc.disable()  # no finalizers of device objects inside the capture (train/graph.py)
        try:
            if unroll:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self.call(model)
                self.graph, self.step_graph = g, None
            else:
                g, gs = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self.prefill(model)
                with torch.cuda.graph(gs, pool=g.pool()):
                    self.step(model)
                self.graph, self.step_graph = g, gs
        finally:
            if was:
                gc.enable()
        return toks

    def _replay(self):
        self.graph.replay()
        if self.step_graph is not None:
            for _ in range(self.max_new - 1):
                self.step_graph.replay()


_GRAPHS = {}
_PINNED = {}


def _pinned(shape, dtype):
    """A reusable page-locked host buffer (pageable copies cost ~100 us each way on this stack:
    profiles/r5/gen_timeline_r5m.txt)."""
    key = (tuple(shape), dtype)
    b = _PINNED.get(key)
    if b is None:
        if len(_PINNED) >= 16:
            _PINNED.pop(next(iter(_PINNED)))
        b = _PINNED[key] = torch.empty(shape, dtype=dtype, pin_memory=torch.cuda.is_available())
    return b


def _to_host(t):
    """int64 host copy of a (small) tensor through a pinned buffer (one DMA, one stream sync)."""
    if t.device.type != "cuda":
        return t.to(torch.long)
    b = _pinned(t.shape, t.dtype)
    b.copy_(t, non_blocking=True)
    torch.cuda.current_stream(t.device).synchronize()
    return b.to(torch.long)


_ARENA_HOLDER = {}


def _arena_version(model):
    """Version of the model's LoRA arena (bumped by every optimizer step / load), None without one.

    The module holding it is remembered per model (a module walk is ~100 Python attribute lookups,
    paid on every graphed call otherwise); a new arena rebinds ``_arena`` on the same modules, so
    reading the remembered module's attribute stays current."""
    ent = _ARENA_HOLDER.get(id(model))
    if ent is not None and ent[0]() is model:
        a = getattr(ent[1], "_arena", None)
        if a is not None:
            return (id(a), a.version)
    for m in model.modules():
        a = getattr(m, "_arena", None)
        if a is not None:
            if len(_ARENA_HOLDER) >= 16:
                _ARENA_HOLDER.pop(next(iter(_ARENA_HOLDER)))
            _ARENA_HOLDER[id(model)] = (weakref.ref(model), m)
            return (id(a), a.version)
    return None


def _decode_graph(model, key_args):
    # Not keyed by the adapter version: every replay rebuilds the LoRA operand packs inside the graph
    # (captured pack launches read the live fp32 arena), so a graph stays valid across optimizer steps
    # and one entry per (model, shape) is kept — the version key made every generate() after a step pay
    # an eager call + a new capture and kept up to 4 stale KV caches / pools resident.
    key = (id(model),) + tuple(key_args[:10])
    for k in [k for k, g in _GRAPHS.items() if g.model_ref() is None or (k[0] == id(model) and g.model_ref() is not model)]:
        _GRAPHS.pop(k)  # dead model, or a new model that reuses a dead one's id()
    g = _GRAPHS.get(key)
    if g is None:
        if len(_GRAPHS) >= 4:
            _GRAPHS.pop(next(iter(_GRAPHS)))
        g = _GRAPHS[key] = _DecodeGraph(model, *key_args)
    return g


@torch.no_grad()
def generate(model, input_ids, attention_mask=None, max_new_tokens=16, eos_token_id=None, pad_token_id=None,
             max_length=None):
    """Greedy decoding.  input_ids [B, S0] (left-padded if ``attention_mask`` has zeros).

    Returns [B, S0 + n_generated] token ids (HF ``generate`` output layout)."""
    if model.training:  # a module walk per call otherwise (the graphed call is host-bound)
        model.eval()
    dev = input_ids.device
    B, S0 = input_ids.shape
    cfg = model.config
    eos = cfg.eos_token_id if eos_token_id is None else eos_token_id
    pad = getattr(cfg, "pad_token_id", eos) if pad_token_id is None else pad_token_id
    if max_length is not None:
        max_new_tokens = max(0, min(max_new_tokens, max_length - S0))
    # the mask's checks run on the host: one small device-to-host copy instead of a chain of tiny
    # kernels and syncs ahead of the (graph-replayed) call
    if attention_mask is None:
        lens_h = torch.full((B,), S0, dtype=torch.long)
        padded = False
    else:
        mk = _to_host(attention_mask).numpy()  # numpy: ~3x less host time than torch CPU ops at this size
        ln = mk.sum(1)
        if (mk != (np.arange(S0)[None, :] >= (S0 - ln)[:, None])).any():
            raise ValueError("generate expects left padding (HF padding_side='left')")
        padded = bool((ln < S0).any())
        lens_h = torch.from_numpy(ln.astype(np.int64))
    fused = model._use_fused(input_ids)
    H, hd = _heads(model)
    emb = model.tied_embedding()
    dtype, vocab = emb.dtype, emb.shape[0]
    fill = pad if pad is not None and 0 <= pad < vocab else 0
    if (fused and dev.type == "cuda" and max_new_tokens > 2 and os.environ.get("MIFT_GEN_GRAPH", "1") != "0"
            and S0 + max_new_tokens <= 16384):
        # the graphed call uploads the prompt lengths itself (pinned); nothing below runs on its path
        dg = _decode_graph(model, (B, S0, max_new_tokens, padded, pad, eos, fill, H, hd, dtype, dev))
        return _graphed_generate(dg, model, input_ids, lens_h, max_new_tokens, eos)
    lens = lens_h.to(dev)
    plen = lens.to(torch.int32).contiguous() if padded else None
    L = len(model.blocks())
    cache = KVCache(L, B, H, S0 + max_new_tokens, hd, dtype, dev)

    # prefill over right-aligned prompts: row b = ids[b, start_b:] then padding, positions 0..S0-1
    start = S0 - lens
    ar = torch.arange(S0, device=dev)
    # filler after each right-aligned prompt / input of a finished row (``fill`` above): any id INSIDE
    # the embedding table.  Filler K/V are masked (kv_len, the decode gap) but still multiplied by
    # p = 0 inside the kernels' P·V, so an out-of-table id (GPT-2's pad = eos = 50256 on a smaller test
    # vocabulary) read garbage rows and a non-finite V turned 0·V into NaN for the whole row.
    if padded:
        src = (ar[None, :] + start[:, None]).clamp(max=S0 - 1)
        ids_r = torch.where(ar[None, :] < lens[:, None], torch.gather(input_ids, 1, src),
                            torch.full_like(input_ids, fill))
    else:
        ids_r = input_ids
    h = model.embed_at(ids_r, ar[None, :].expand(B, S0).contiguous())
    h = _run_blocks(model, h, lambda li: _prefill_attn(cache, li, B, S0, H, hd, plen, fused), fused)
    last = (lens - 1).clamp(min=0)
    h_last = torch.gather(h, 1, last[:, None, None].expand(B, 1, h.shape[-1])) if padded else h[:, -1:]
    logits = model.head_logits(h_last)
    nxt = logits[:, -1].float().argmax(-1)
    out = [input_ids]
    done = torch.zeros(B, dtype=torch.bool, device=dev)
    for i in range(max_new_tokens):
        nxt = torch.where(done, torch.full_like(nxt, pad), nxt)
        out.append(nxt[:, None])
        if eos is not None:
            done = done | (nxt == eos)
        if i == max_new_tokens - 1 or (eos is not None and bool(done.all())):
            break
        t = S0 + i
        pos = (lens + i)[:, None]
        h = model.embed_at(torch.where(done, torch.full_like(nxt, fill), nxt)[:, None], pos)
        h = _run_blocks(model, h, lambda li: _decode_attn(cache, li, B, H, hd, t, plen, S0, fused), fused)
        nxt = model.head_logits(h)[:, -1].float().argmax(-1)
    return torch.cat(out, 1)


def _graphed_generate(dg, model, input_ids, lens, max_new_tokens, eos):
    """The whole call from one graph replay (or its eager first run); HF's early stop applied after."""
    toks = dg.run(model, input_ids, lens).clone()
    if eos is not None and eos >= 0:  # (a negative id is never emitted)
        # HF stops after the step in which the last unfinished row emitted EOS
        hit = toks == eos
        if bool(hit.any(1).all()):
            first = torch.where(hit, torch.arange(max_new_tokens, device=toks.device)[None, :],
                                max_new_tokens).min(1).values
            toks = toks[:, :int(first.max()) + 1]
    return torch.cat([input_ids, toks], 1)


@torch.no_grad()
def generate_nocache(model, input_ids, max_new_tokens=16):
    """Oracle: re-run the full forward for every new token (unpadded input only)."""
    ids = input_ids
    for _ in range(max_new_tokens):
        logits = model(input_ids=ids)["logits"]
        ids = torch.cat([ids, logits[:, -1].float().argmax(-1, keepdim=True)], 1)
    return ids
