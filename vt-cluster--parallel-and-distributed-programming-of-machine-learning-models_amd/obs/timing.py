"""Reference-format timing / step logs.

Formats (kept verbatim so the reference's summarizers and ``eval_logs.py``
parse our logs unchanged — SURVEY Appendix A.3/A.4):
  * ``timing_rank{r}.log``: first line ``Timings (sec)`` then ``[<Phase>] <s:.2f> sec``
    (``P1/finetune_lora_distilgpt2.py:56-65``); stdout ``[{host}] rank={r} ⏱ {phase}: {s:.2f}s``.
  * P1 StepTimer: ``[{host}] rank={r} step {N} {s:.3f}s`` (``P1/...:117-122``).
  * tiny-lab StepTimer: ``[rank {r} | step {N}] step_ms=… samples_per_sec=… tokens_per_sec=…``
    (``labs/tiny/train_tiny.py:70-86``).
  * P2 loss line: ``[R{rank}] ep={e} step={s} loss={l:.4f} (+{t:.1f}s)`` (``P2/...:221-224``).
"""
import json
import os
import socket
import time

HOST = socket.gethostname()


class PhaseLogger:
    def __init__(self, logdir: str, rank: int, fresh: bool = True):
        self.logdir, self.rank = logdir, rank
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"timing_rank{rank}.log")
        if fresh:
            with open(self.path, "w") as f:
                f.write("Timings (sec)\n")

    def log(self, phase: str, seconds: float, echo: bool = True):
        with open(self.path, "a") as f:
            f.write(f"[{phase}] {seconds:.2f} sec\n")
        if echo:
            print(f"[{HOST}] rank={self.rank} ⏱ {phase}: {seconds:.2f}s", flush=True)

    def phase(self, name: str):
        return _Phase(self, name)


class _Phase:
    def __init__(self, lg, name):
        self.lg, self.name = lg, name

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.seconds = time.perf_counter() - self.t0
        self.lg.log(self.name, self.seconds)


def p1_step_line(rank, step, seconds):
    return f"[{HOST}] rank={rank} step {step} {seconds:.3f}s"


def lab_step_line(rank, step, step_ms, samples_per_sec, tokens_per_sec):
    return (f"[rank {rank} | step {step}] step_ms={step_ms:.2f} samples_per_sec={samples_per_sec:.2f} "
            f"tokens_per_sec={tokens_per_sec:.2f}")


def p2_loss_line(rank, ep, step, loss, dt):
    return f"[R{rank}] ep={ep} step={step} loss={loss:.4f} (+{dt:.1f}s)"


def perf_line(rank, step, tokens_per_sec, tflops, hbm_gb, comm_ms, world):
    """MI355X additions to the reference metrics: whole-job padded tokens/s, model
    TFLOP/s per GPU (6·N·T-style estimate, LoRA: no base weight grads), peak HBM per rank and the
    gradient all-reduce time of the last step."""
    return (f"[perf] rank={rank} step={step} world={world} tokens_per_sec={tokens_per_sec:.1f} "
            f"tflops_per_gpu={tflops:.1f} hbm_gb={hbm_gb:.2f} comm_ms={comm_ms:.3f}")


def hf_log_line(d: dict):
    """Trainer-style ``{'loss': ..., 'learning_rate': ..., 'epoch': ...}``."""
    return str({k: (round(v, 4) if (isinstance(v, float) and k in ("loss", "grad_norm", "epoch")) else v)
                for k, v in d.items()})


def write_json(path, obj):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(obj, f, indent=2)
