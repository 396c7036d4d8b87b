"""Fault injection for teardown / resume tests (SURVEY §5.3 plan).

``MIFT_FAULT=rank:step:kind[:where]`` — on global rank ``rank`` (``*`` = all) when the
trainer reaches optimizer step ``step``: ``raise`` (RuntimeError), ``exit``
(os._exit(17), like a killed node) or ``hang`` (sleep until the collective
timeout / watchdog fires).  ``where`` is ``step`` (after the optimizer
step, default) or ``micro`` (inside the micro-batch loop).  Used only by
tests; a no-op when the variable is unset.
"""
import os
import time

EXIT_CODE = 17
_fired = False


def parse(spec: str):
    parts = spec.split(":")
    if len(parts) < 3:
        raise ValueError(f"bad MIFT_FAULT spec {spec!r}")
    where = parts[3] if len(parts) > 3 else "step"
    return (None if parts[0] == "*" else int(parts[0])), int(parts[1]), parts[2], where


def maybe_inject(rank: int, step: int, where: str = "step", grads=None):
    spec = os.environ.get("MIFT_FAULT")
    if not spec:
        return
    global _fired
    r, s, kind, w = parse(spec)
    if _fired or (r is not None and r != rank) or s != step or w != where:
        return
    if kind == "inf" and grads is None:
        return
    _fired = True  # once per process (several micro-batches share a step number)
    print(f"[FAULT] injecting {kind} on rank {rank} at step {step} ({where})", flush=True)
    if kind == "inf":
        grads.view(-1)[0] = float("inf")
        return
    if kind == "raise":
        raise RuntimeError(f"injected fault on rank {rank} step {step}")
    if kind == "exit":
        os._exit(EXIT_CODE)
    if kind == "hang":
        time.sleep(float(os.environ.get("MIFT_FAULT_HANG_S", "3600")))
        return
    raise ValueError(f"unknown fault kind {kind}")
