"""Side HIP stream for off-critical-path backward work.

The LoRA weight gradients (dA, dB: ``lora_wgrad`` into the flat fp32 grad
arena) are consumed only by the optimizer / gradient all-reduce at the end of
the step, while the dgrad chain that follows them is the critical path.  They
therefore run on a second stream: each launch waits (device-side event) for
the main stream to have produced its inputs, the inputs are tagged with
``record_stream`` so the caching allocator keeps them alive, and the first
launch of a backward pass queues an autograd-engine callback that makes the
issuing stream wait for the side stream when ``backward()`` finishes — so
everything after backward (grad-norm, RCCL all-reduce, AdamW) sees complete
gradients with no host synchronisation.  The small wgrad kernels then fill
CUs left idle by the dgrad GEMMs instead of serialising between them.

The per-launch event traffic costs host time, so in eager mode the side
stream only pays when the host runs ahead of the GPU; under hipGraph capture
(mift.train.graph) the fork/join becomes graph edges and costs nothing per
replay.  ``MIFT_SIDE_STREAM=0`` runs the work inline; ``set_enabled``
overrides per process (the graphed trainer turns it on).
"""
import os

import torch

_SIDE = {}
_STATE = {"enabled": os.environ.get("MIFT_SIDE_STREAM", "auto")}


def set_enabled(on):
    """True / False / None (None = environment default)."""
    _STATE["enabled"] = os.environ.get("MIFT_SIDE_STREAM", "auto") if on is None else ("1" if on else "0")


def enabled():
    v = _STATE["enabled"]
    if v == "auto":  # eager default: inline (event traffic would make the host the bottleneck)
        return False
    return v != "0"


class _Side:
    __slots__ = ("stream", "main", "pending")

    def __init__(self, dev):
        self.stream = torch.cuda.Stream(device=dev)
        self.main = None
        self.pending = False


def _join_all():
    for ent in _SIDE.values():
        if ent.pending:
            ent.main.wait_stream(ent.stream)
            ent.pending = False


def run_side(dev, fn, *tensors):
    """Run ``fn()`` (kernel launches) on the side stream of ``dev`` after the
    work already queued on the current stream; keep ``tensors`` alive."""
    if not enabled() or not torch.cuda.is_available():
        fn()
        return
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    ent = _SIDE.get(idx)
    if ent is None:
        ent = _SIDE[idx] = _Side(torch.device("cuda", idx))
    cur = torch.cuda.current_stream(idx)
    if ent.pending and ent.main != cur:
        _join_all()
    ent.stream.wait_stream(cur)
    with torch.cuda.stream(ent.stream):
        fn()
    for t in tensors:
        if t is not None:
            t.record_stream(ent.stream)
    if not ent.pending:
        ent.pending, ent.main = True, cur
        try:
            torch.autograd.Variable._execution_engine.queue_callback(_join_all)
        except RuntimeError:
            pass  # not inside a backward pass: joined by the next explicit join()


def join():
    """Make the issuing streams wait for all side-stream work (idempotent)."""
    _join_all()
