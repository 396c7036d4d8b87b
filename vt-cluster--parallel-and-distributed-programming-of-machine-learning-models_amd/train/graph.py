"""hipGraph capture of the training step (MI355X: HIP graphs instead of a tracing compiler).

A distilgpt2 LoRA optimizer step is ~250 kernel launches in ~6 ms of GPU
time; issuing them from Python through autograd costs ~2.8 ms of host time
per step (tools/graph_overhead.py), 0.17 ms as a graph replay.  The eager
step is therefore GPU-bound today, but the host cost becomes the limit as the
kernels get faster, with more micro-batches per step, and for small decode
steps.  ``GraphedStep`` captures the forward and
backward of all micro-batches of a step — LoRA packing, fused kernels, the
hand-written fused LM head + cross-entropy — into ONE hipGraph and replays it: one host launch per
step and no inter-kernel gaps.  ``MIFT_GRAPH_SIDE=1`` also forks the LoRA
weight-gradient kernels onto a side stream inside the graph (mift.ops.streams);
measured on MI355X it slows the co-running dgrad GEMMs more than it hides
(device 6.18 vs 5.99 ms/step, tools/graph_overhead.py), so it is off.

What stays outside the graph (per step, on the host stream):
  * staging the micro-batches into the graph's static input buffers
    (async copies from pinned host memory);
  * the per-step scalars as device tensors: 1/global-token-count and the
    micro-step counters that every dropout kernel mixes into its seed
    (``mift_seed`` in csrc/common.h; ``dropout_seed`` in models/layers.py) —
    so replays draw fresh masks, bit-identical to the eager path;
  * the DP gradient all-reduce (RCCL), the grad-norm / clip / AdamW kernels
    and the LR update: a handful of launches, kept eager so collectives are
    never captured.

Captures are keyed by the micro-batch shapes (the last, shorter step of an
epoch gets its own graph or runs eagerly); the first step of every shape runs
eagerly as warm-up (lazy library init, workspace allocation).
"""
import gc
import os

import torch

from ..models.layers import graph_seeds
from ..ops import streams


class GraphedStep:
    def __init__(self, trainer, max_graphs: int = 3):
        self.tr = trainer
        self.graphs = {}      # signature -> dict(graph, static, steps_t, loss)
        self.seen = set()     # signatures already run eagerly once (warm-up)
        self.max_graphs = max_graphs
        self.pool = None

    @staticmethod
    def signature(mbs):
        return tuple((k, tuple(v.shape), v.dtype) for mb in mbs for k, v in sorted(mb.items()))

    def supported(self, mbs):
        sig = self.signature(mbs)
        if sig in self.graphs:
            return True
        if sig not in self.seen:
            self.seen.add(sig)
            return False  # eager warm-up for this shape
        return len(self.graphs) < self.max_graphs

    def prepare(self, mbs):
        """Capture the graph for this shape right after its eager warm-up step, so the capture's
        host cost lands in that step and the NEXT step already replays (a benchmark with one
        warm-up step then times replays only)."""
        sig = self.signature(mbs)
        if sig in self.seen and sig not in self.graphs and len(self.graphs) < self.max_graphs:
            self._capture(sig, mbs)

    # ------------------------------------------------------------------
    def _fwd_bwd(self, ent, n):
        """The captured region: forward + backward of every micro-batch.  Returns the step's summed
        loss — a tensor of the graph's pool that every replay rewrites (no copy kernel)."""
        tr, model = self.tr, self.tr.model
        C = _C()
        from ..ops import fused
        gscale = None
        acc = None
        for i in range(n):
            C.set_seed_step(ent["steps_t"][i:i + 1])
            mb = ent["static"][i]
            # the fused LM head multiplies its upstream grad by 1/tokens inside its dgrad reduction,
            # so backward is seeded with the loss scale itself: no scalar multiply kernel per step
            fused.set_head_grad_mul(ent["inv_ntok"])
            try:
                out = model(input_ids=mb["input_ids"], attention_mask=mb["attention_mask"], labels=mb["labels"],
                            reduction="sum", return_logits=False)
                used = fused.head_grad_mul_used()
            finally:
                fused.set_head_grad_mul(None)
            loss_sum = out["loss"].float()
            if used:
                seed = tr.opt.loss_scale_t.reshape(())
            else:  # a head without the multiplier (library / classification heads)
                if gscale is None:
                    gscale = (tr.opt.loss_scale_t * ent["inv_ntok"]).reshape(())
                seed = gscale
            loss_sum.backward(seed)
            streams.join()
            acc = loss_sum.detach() if acc is None else acc + loss_sum.detach()
        C.set_seed_step(None)
        return acc

    # Per-step inputs of a replay — every micro-batch tensor, the micro-step counters and 1/tokens —
    # live in ONE device buffer that one async copy refreshes from a ring of pinned staging buffers
    # (host-side packing): one SDMA transfer per step instead of three per micro-batch + two scalar
    # kernels (the separate transfers left a ~40 us hole at the top of every replayed step).
    _RING = 4

    def _layout(self, mbs):
        items, off = [], 0
        for i, mb in enumerate(mbs):
            for k, v in sorted(mb.items()):
                n = v.numel() * v.element_size()
                items.append((i, k, off, n, v.dtype, tuple(v.shape)))
                off = (off + n + 255) // 256 * 256
        steps_off = off
        off = (off + 8 * len(mbs) + 255) // 256 * 256
        return items, steps_off, off, off + 4  # ..., inv_ntok offset, total bytes

    def _capture(self, sig, mbs):
        tr, model = self.tr, self.tr.model
        dev = tr.device
        items, steps_off, inv_off, total = self._layout(mbs)
        dbuf = torch.zeros(total, dtype=torch.uint8, device=dev)
        static = [dict() for _ in mbs]
        for i, k, off, n, dt, shp in items:
            static[i][k] = dbuf[off:off + n].view(dt).view(shp)
        pin = torch.cuda.is_available()
        ent = {"static": static, "loss": None,
               "steps_t": dbuf[steps_off:steps_off + 8 * len(mbs)].view(torch.int64),
               "inv_ntok": dbuf[inv_off:inv_off + 4].view(torch.float32),
               "dbuf": dbuf, "items": items, "steps_off": steps_off, "inv_off": inv_off,
               "stage": [torch.zeros(total, dtype=torch.uint8, pin_memory=pin) for _ in range(self._RING)],
               "stage_ev": [None] * self._RING, "slot": 0}
        for i, mb in enumerate(mbs):
            for k, v in mb.items():
                static[i][k].copy_(v)
        # force the per-step LoRA operand packing into the captured region
        from ..ops.fused import invalidate_packs
        invalidate_packs(model)
        g = torch.cuda.CUDAGraph()
        ms0 = model.micro_step
        torch.cuda.synchronize()
        graph_seeds(True)
        streams.set_enabled(os.environ.get("MIFT_GRAPH_SIDE", "0") == "1")
        red = tr.reducer
        # no Python GC inside the capture: torch.cuda.graph collects once at entry, but a collection
        # triggered mid-capture ran finalizers of device objects and aborted the process (seen once
        # in tests/test_graph_gpu.py, GC-timing dependent)
        gc_was = gc.isenabled()
        gc.disable()
        try:
            # collectives are never captured: the DP buckets launch after the replay (finish())
            with (red.no_sync() if red is not None else _nullctx()):
                with torch.cuda.graph(g, pool=self.pool, capture_error_mode="thread_local"):
                    ent["loss"] = self._fwd_bwd(ent, len(mbs))
        finally:
            if gc_was:
                gc.enable()
            graph_seeds(False)
            streams.set_enabled(None)
            _C().set_seed_step(None)
            model.micro_step = ms0
        if self.pool is None:
            self.pool = g.pool()
        ent["graph"] = g
        self.graphs[sig] = ent
        return ent

    # ------------------------------------------------------------------
    def run(self, mbs, ntok):
        """Forward + backward of one optimizer step by graph replay; returns the summed loss tensor."""
        tr, model = self.tr, self.tr.model
        sig = self.signature(mbs)
        ent = self.graphs.get(sig)
        fresh = ent is None
        if fresh:
            ent = self._capture(sig, mbs)
        n = len(mbs)
        slot = ent["slot"]
        ent["slot"] = (slot + 1) % self._RING
        ev = ent["stage_ev"][slot]
        if ev is not None:
            ev.synchronize()  # that staging buffer's previous upload has been consumed
        st = ent["stage"][slot]
        for i, k, off, nb, dt, shp in ent["items"]:
            st[off:off + nb].view(dt).view(shp).copy_(mbs[i][k])
        st[ent["steps_off"]:ent["steps_off"] + 8 * n].view(torch.int64).copy_(
            torch.arange(model.micro_step + 1, model.micro_step + n + 1, dtype=torch.int64))
        st[ent["inv_off"]:ent["inv_off"] + 4].view(torch.float32).fill_(1.0 / float(ntok))
        ent["dbuf"].copy_(st, non_blocking=True)
        if ent["stage_ev"][slot] is None:
            ent["stage_ev"][slot] = torch.cuda.Event()
        ent["stage_ev"][slot].record()
        ent["graph"].replay()
        model.micro_step += n
        return ent["loss"]


def _C():
    from ..ops.dispatch import C
    return C()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
