"""Step-window profiler for the training apps (SURVEY §5.1 "Tracing / profiling").

The reference has no profiler; its only timing is the phase log and per-step wall clock
(``Cluster/Project 1 - Fine Tuning Distilgpt2/finetune_lora_distilgpt2.py:56-65``, ``:117-122``).
Here ``--profile DIR [--profile_steps A:B]`` on the P1/P2 apps (``TrainConfig.profile_dir``)
records optimizer steps [A, B) of every rank with ``torch.profiler`` (host ops + HIP kernels)
and writes per rank:

  * ``DIR/trace_rank{r}.json``  — Chrome/Perfetto trace (kernels, memcpy, RCCL kernels);
  * ``DIR/kernels_rank{r}.txt`` — top device-time table;
  * ``DIR/ranges_rank{r}.json`` — wall-clock (host) ms of each named range per step.

Named ranges are emitted by the engine with :func:`rng` — ``mift.step``, ``mift.fwd_bwd``,
``mift.comm.bucket{i}`` (one per DDP gradient bucket, tagged backward/finish),
``mift.comm.zero_rs`` / ``mift.comm.zero_ag``, ``mift.pp.send`` / ``mift.pp.recv``,
``mift.optimizer``.  They are ``torch.profiler.record_function`` ranges, so they appear in the
trace, and with ``MIFT_ROCTX=1`` they are also pushed as ROCTX markers
(``torch.cuda.nvtx`` is roctx on ROCm) for ``rocprofv3 --marker-trace``.

Outside a profiled window :func:`rng` costs one attribute check.
"""
import contextlib
import json
import os
import time

_ACTIVE = False
_ROCTX = os.environ.get("MIFT_ROCTX", "0") == "1"
_ranges = None  # name -> list of host ms, while a window is recording


@contextlib.contextmanager
def rng(name):
    """Named range: recorded only while a profiling window is open (or MIFT_ROCTX=1)."""
    if not _ACTIVE and not _ROCTX:
        yield
        return
    import torch
    pushed = False
    if _ROCTX and torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        pushed = True
    t0 = time.perf_counter()
    try:
        if _ACTIVE:
            with torch.profiler.record_function(name):
                yield
        else:
            yield
    finally:
        if _ranges is not None:
            _ranges.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
        if pushed:
            torch.cuda.nvtx.range_pop()


def parse_window(spec, default=(3, 6)):
    """'A:B' -> (A, B) optimizer steps (1-based global steps, B exclusive); '' -> default."""
    if not spec:
        return default
    a, _, b = str(spec).partition(":")
    a = int(a)
    b = int(b) if b else a + 3
    if a < 1 or b <= a:
        raise ValueError(f"profile window must be A:B with 1 <= A < B, got {spec!r}")
    return a, b


class StepProfiler:
    """Opens a torch.profiler window over global steps [start, stop) and dumps it per rank."""

    def __init__(self, out_dir, rank, window=(3, 6)):
        self.out_dir, self.rank = out_dir, rank
        self.start, self.stop = window
        self.prof = None
        self.done = False

    def before_step(self, step):
        """``step`` = the 1-based global step about to run."""
        global _ACTIVE, _ranges
        if self.done or self.prof is not None or step != self.start:
            return
        import torch
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
            torch.cuda.synchronize()
        self.prof = torch.profiler.profile(activities=acts, record_shapes=False, with_stack=False)
        self.prof.__enter__()
        _ACTIVE, _ranges = True, {}

    def after_step(self, step):
        """``step`` = the 1-based global step that just finished."""
        if self.prof is None or step + 1 < self.stop:
            return
        self.close()

    def close(self):
        global _ACTIVE, _ranges
        if self.prof is None:
            return
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.prof.__exit__(None, None, None)
        ranges, _ACTIVE, _ranges = _ranges or {}, False, None
        os.makedirs(self.out_dir, exist_ok=True)
        r = self.rank
        self.prof.export_chrome_trace(os.path.join(self.out_dir, f"trace_rank{r}.json"))
        key = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
        with open(os.path.join(self.out_dir, f"kernels_rank{r}.txt"), "w") as f:
            f.write(self.prof.key_averages().table(sort_by=key, row_limit=40))
        summary = {"rank": r, "steps": [self.start, self.stop],
                   "ranges_ms": {k: {"n": len(v), "total": round(sum(v), 3), "mean": round(sum(v) / len(v), 4)}
                                 for k, v in sorted(ranges.items())}}
        with open(os.path.join(self.out_dir, f"ranges_rank{r}.json"), "w") as f:
            json.dump(summary, f, indent=1)
        self.prof, self.done = None, True
