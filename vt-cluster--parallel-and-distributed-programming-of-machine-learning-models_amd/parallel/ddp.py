"""Data-parallel gradient reduction over the flat LoRA arena (RCCL over xGMI).

Replaces HF Trainer -> torch DDP (reference C16, X6/X7) with a design sized
for LoRA on MI355X:
  * no parameter broadcast at construction: every rank builds identical
    weights from the same seed / file, and ``verify_replicas`` checks a
    checksum (all-reduce of MAX-MIN) instead of broadcasting 329 MB (X6);
  * the gradient arena is split into buckets in *reverse* module order; a
    post-accumulate-grad hook counts readiness and launches each bucket's
    async all-reduce (SUM — the loss is already normalised by the global
    token count) as soon as its last tensor is done, overlapping the rest
    of backward; ``finish()`` waits for all handles;
  * ``no_sync()`` for accumulation micro-steps (reference ``no_sync`` on
    steps 1..accum-1, verified in SURVEY C16);
  * default bucket 25 MB: distilgpt2 LoRA (1.6 MB fp32) and OPT-2.7B
    (47 MB, 11.8 MB per PP stage) are latency-bound on xGMI, so one or two
    buckets — one-shot all-reduce in RCCL — beat many small ones.
"""
import contextlib

import torch
import torch.distributed as dist


class GradReducer:
    def __init__(self, arena, group=None, bucket_mb: float = 25.0, overlap: bool = True, world: int = None):
        self.arena = arena
        self.group = group
        self.world = world if world is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
        self.enabled = self.world > 1
        self.overlap = overlap and self.enabled
        self._sync = True
        self.handles = []
        # buckets over reverse module order (backward produces last layers first)
        cap = int(bucket_mb * 1024 * 1024 / 4)
        named = list(zip(arena.named, arena.offsets))
        buckets, cur, cur_n = [], [], 0
        for (n, p), off in reversed(named):
            cur.append((p, off))
            cur_n += p.numel()
            if cur_n >= cap:
                buckets.append(cur)
                cur, cur_n = [], 0
        if cur:
            buckets.append(cur)
        self.buckets = []
        for b in buckets:
            lo = min(off for _, off in b)
            hi = max(off + p.numel() for p, off in b)
            self.buckets.append({"params": [p for p, _ in b], "lo": lo, "hi": hi, "pending": len(b)})
        self._p2b = {}
        for i, b in enumerate(self.buckets):
            for p in b["params"]:
                self._p2b[id(p)] = i
        self._hooks = []
        if self.overlap:
            for _, p in arena.named:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    def _launch(self, b):
        sl = self.arena.grad[b["lo"]:b["hi"]]
        self.handles.append(dist.all_reduce(sl, group=self.group, async_op=True))

    def _on_grad(self, p):
        if not self._sync or not self.overlap:
            return
        b = self.buckets[self._p2b[id(p)]]
        b["pending"] -= 1
        if b["pending"] == 0:
            self._launch(b)

    def finish(self):
        """Call after the last micro-batch's backward of an optimizer step."""
        if not self.enabled:
            return
        if self.overlap:
            for b in self.buckets:
                if b["pending"] > 0:  # params that got no grad this step (unused) -> launch anyway
                    self._launch(b)
        else:
            for b in self.buckets:
                self._launch(b)
        for h in self.handles:
            h.wait()
        self.handles = []
        for b in self.buckets:
            b["pending"] = len(b["params"])

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


@torch.no_grad()
def verify_replicas(tensors, group=None, atol=0.0):
    """Checksum every tensor across the group; raise if replicas diverge.

    Replaces DDP's construction-time broadcast: identical init by seed,
    verified with one all-reduce of [max, -min] of per-tensor sums."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return True
    sums = torch.stack([t.detach().float().sum() for t in tensors])
    mx = sums.clone()
    mn = -sums.clone()
    both = torch.stack([mx, mn])
    dist.all_reduce(both, op=dist.ReduceOp.MAX, group=group)
    spread = (both[0] + both[1]).abs().max().item()
    if spread > atol + 1e-3 * sums.abs().max().item():
        raise RuntimeError(f"replica divergence detected: max checksum spread {spread}")
    return True
