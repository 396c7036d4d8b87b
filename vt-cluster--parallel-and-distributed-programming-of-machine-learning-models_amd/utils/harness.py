"""Multi-process rehearsal harness: run ``fn(rank, world, **kw)`` in ``world``
spawned processes with the env:// contract set (127.0.0.1 rendezvous, gloo on
CPU), collect each rank's return value.  Used by the CPU test-suite to cover
DDP / PP / DP×PP / ZeRO-1 with world_size > 1 without GPUs, and usable on a
single-GPU box to rehearse RCCL-free multi-rank runs.
"""
import os
import pickle
import socket
import tempfile
import traceback

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, kw, outdir, env):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "MIFT_DEVICE": "cpu"})
    os.environ.update(env or {})
    import torch
    torch.set_num_threads(1)
    try:
        res = fn(rank, world, **kw)
        err = None
    except Exception:  # noqa: BLE001 - reported to the parent
        res, err = None, traceback.format_exc()
    with open(os.path.join(outdir, f"rank{rank}.pkl"), "wb") as f:
        pickle.dump((res, err), f)
    if err:
        raise SystemExit(1)


def run(fn, world, env=None, timeout=300, **kw):
    """-> [result of rank 0, ..., rank world-1]; raises with the first rank's traceback."""
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_entry, args=(r, world, port, fn, kw, d, env)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout)
        for p in procs:
            if p.is_alive():
                p.kill()
        out = []
        for r in range(world):
            path = os.path.join(d, f"rank{r}.pkl")
            if not os.path.exists(path):
                raise RuntimeError(f"rank {r} produced no result (exit {procs[r].exitcode})")
            with open(path, "rb") as f:
                res, err = pickle.load(f)  # our own children's output
            if err:
                raise RuntimeError(f"rank {r} failed:\n{err}")
            out.append(res)
        return out
