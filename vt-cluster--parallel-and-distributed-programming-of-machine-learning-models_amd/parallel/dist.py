"""Distributed bring-up: env:// contract, SLURM fallbacks, device binding, DP×PP grid.

Reference parity:
  * ``utils/parallel_utils.py:17-57`` — ``init_distributed(local_rank)``,
    ``world_size()``, ``is_main_process()``; single-process runs still form a
    world_size=1 gloo group so the code path is identical;
  * ``P1/finetune_lora_distilgpt2.py:35-54`` — env:// init + the 4-byte
    all-reduce "collective OK" sanity check;
  * ``P2/finetune_lora_opt_pp.py:38-54`` — RANK/WORLD_SIZE/LOCAL_RANK with
    SLURM_PROCID/SLURM_NTASKS/SLURM_LOCALID fallbacks (we also fall back for
    RANK, fixing defect B6), ``PIPELINE_PARALLEL_SIZE``.

MI355X-first: one process per GPU; the hot-path group is RCCL (torch backend
"nccl" is RCCL on ROCm) over xGMI; a Gloo group is kept as control plane
(barriers with timeouts, object gathers, CPU-only runs).  The rendezvous is
the c10d TCPStore at MASTER_ADDR:MASTER_PORT, unchanged from the reference.
"""
import datetime
import os
import socket
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return int(v)
    return default


def _first_slurm_host():
    nl = os.environ.get("SLURM_JOB_NODELIST") or os.environ.get("SLURM_NODELIST")
    if not nl:
        return None
    # expand the first entry of e.g. "hpc[12-15,20],gpu3"
    head = nl.split(",")[0]
    if "[" in head:
        pre, rng = head.split("[", 1)
        first = rng.rstrip("]").split(",")[0].split("-")[0]
        return pre + first
    return head


def env_rank_info():
    """(rank, world, local_rank) from torchrun env, else SLURM, else single."""
    rank = _env_int("RANK", "SLURM_PROCID", default=0)
    world = _env_int("WORLD_SIZE", "SLURM_NTASKS", default=1)
    local = _env_int("LOCAL_RANK", "SLURM_LOCALID", default=0)
    return rank, world, local


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "gloo"
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    master: str = "127.0.0.1:29500"
    ctrl_group: Optional[object] = None     # gloo control plane
    # grid
    dp: int = 1
    pp: int = 1
    dp_rank: int = 0
    pp_rank: int = 0
    dp_group: Optional[object] = None
    pp_group: Optional[object] = None
    pp_ranks: List[int] = field(default_factory=list)
    timeout: Optional[object] = None        # collective timeout (watchdog) for every group
    dp_ranks: List[int] = field(default_factory=list)
    pp_fwd_group: Optional[object] = None   # p2p (MIFT_PP_P2P=shared): activations, whole replica
    pp_bwd_group: Optional[object] = None   # p2p (MIFT_PP_P2P=shared): activation grads, whole replica
    # p2p (default MIFT_PP_P2P=link): one 2-rank communicator per adjacent stage pair AND direction:
    # link_*[0] is the link to the previous stage, link_*[1] to the next (None at the ends)
    link_f: List[Optional[object]] = field(default_factory=lambda: [None, None])  # activations s -> s+1
    link_b: List[Optional[object]] = field(default_factory=lambda: [None, None])  # grads s+1 -> s
    # interleaved pipeline (pp_virtual > 1 model chunks per rank): the wrap-around pair (last stage,
    # first stage) carries chunk c's activations from the last stage to chunk c+1 on the first stage
    # (wrap_f) and the matching gradients back (wrap_b)
    pp_virtual: int = 1
    wrap_f: Optional[object] = None
    wrap_b: Optional[object] = None

    @property
    def is_main(self):
        return self.rank == 0

    @property
    def is_first_stage(self):
        return self.pp_rank == 0

    @property
    def is_last_stage(self):
        return self.pp_rank == self.pp - 1

    def stage_rank(self, stage):
        """Global rank of pipeline `stage` in my replica."""
        return self.pp_ranks[stage]


_CTX: Optional[DistContext] = None


def want_gpu() -> bool:
    if os.environ.get("MIFT_DEVICE", "").lower() == "cpu":
        return False
    try:
        return torch.cuda.device_count() > 0 and torch.cuda.is_available()
    except Exception:
        return False


def init(pp: Optional[int] = None, backend: Optional[str] = None, timeout_s: Optional[int] = None,
         sanity: bool = True, verbose: bool = True, virtual: Optional[int] = None) -> DistContext:
    """Initialise the process group (idempotent) and build the DP×PP grid.

    ``pp`` defaults to $PIPELINE_PARALLEL_SIZE or 1.  Ranks are laid out
    pipeline-major: replica r owns ranks [r*pp, (r+1)*pp).  ``virtual`` (default
    $PIPELINE_VIRTUAL_STAGES or 1): model chunks per pipeline rank (interleaved 1F1B).
    """
    global _CTX
    if _CTX is not None:
        return _CTX
    rank, world, local = env_rank_info()
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(world))
    os.environ.setdefault("LOCAL_RANK", str(local))
    os.environ.setdefault("MASTER_ADDR", _first_slurm_host() or "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    gpu = want_gpu()
    if backend is None:
        backend = os.environ.get("MIFT_BACKEND") or ("nccl" if gpu else "gloo")
    if backend == "nccl" and not gpu:
        backend = "gloo"
    if gpu:
        dev_idx = local % torch.cuda.device_count()
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    timeout = datetime.timedelta(seconds=timeout_s or int(os.environ.get("MIFT_COMM_TIMEOUT",
                                                                         os.environ.get("GLOO_SOCKET_TIMEOUT", "1800"))))
    # RCCL watchdog: a collective that exceeds `timeout` aborts the communicator and
    # tears the process down (non-zero exit -> torchrun / srun --kill-on-bad-exit end the job)
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if not dist.is_initialized():
        kw = dict(backend=backend, init_method="env://", rank=rank, world_size=world, timeout=timeout)
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    ctrl = dist.new_group(backend="gloo", timeout=timeout) if backend != "gloo" else dist.group.WORLD
    ctx = DistContext(rank=rank, world=world, local_rank=local, backend=backend, device=device,
                      master=f"{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}", ctrl_group=ctrl)
    pp = pp or int(os.environ.get("PIPELINE_PARALLEL_SIZE", "1") or 1)
    if pp < 1 or world % pp != 0:
        raise ValueError(f"pipeline size {pp} must divide world size {world}")
    ctx.timeout = timeout
    virtual = virtual or int(os.environ.get("PIPELINE_VIRTUAL_STAGES", "1") or 1)
    if virtual < 1:
        raise ValueError(f"virtual pipeline stages {virtual} < 1")
    build_grid(ctx, pp, virtual)
    _CTX = ctx
    if verbose:
        print(f"[RANK {rank}] WORLD_SIZE={world}", flush=True)
        if rank == 0:
            print(f"[DDP] world={world} master={ctx.master} backend={backend} grid=dp{ctx.dp}xpp{ctx.pp}", flush=True)
    if sanity:
        x = torch.ones(1, device=device)
        dist.all_reduce(x)
        if rank == 0 and verbose:
            print(f"[DDP] collective OK: sum={x.item()} world={world}", flush=True)
    return ctx


def build_grid(ctx: DistContext, pp: int, virtual: int = 1):
    world = ctx.world
    dp = world // pp
    ctx.dp, ctx.pp = dp, pp
    ctx.pp_virtual = virtual if pp > 1 else 1
    ctx.dp_rank, ctx.pp_rank = ctx.rank // pp, ctx.rank % pp
    # only the p2p communicators the selected layout uses are created: under RCCL with a bound
    # device_id every group is a live communicator with its own buffers and streams
    mode = os.environ.get("MIFT_PP_P2P", "link")
    if mode not in ("link", "shared", "blocking"):
        raise ValueError(f"MIFT_PP_P2P={mode!r}: link | shared | blocking")
    ctx.p2p_mode = mode
    ctx.n_groups = 0

    def new_group(ranks):
        ctx.n_groups += 1
        return dist.new_group(ranks, timeout=ctx.timeout)

    # every rank must create every group in the same order
    for r in range(dp):
        ranks = list(range(r * pp, (r + 1) * pp))
        multi = pp > 1 and world > 1
        g = new_group(ranks) if multi else None  # grad-norm / found-inf / loss reductions over the pipe
        if ctx.rank in ranks:
            ctx.pp_group, ctx.pp_ranks = g, ranks
        if multi and mode == "shared":
            # replica-wide p2p communicators per direction (the round-2 layout)
            gf, gb = new_group(ranks), new_group(ranks)
            if ctx.rank in ranks:
                ctx.pp_fwd_group, ctx.pp_bwd_group = gf, gb
        # per-link communicators (link / blocking): stage s's "recv from s-1" and "send to s+1" are on
        # different communicators, hence different RCCL streams, so neither ever queues behind the
        # other (pipeline.py, "p2p ordering")
        for s in range(pp - 1) if (multi and mode != "shared") else ():
            pair = [ranks[s], ranks[s + 1]]
            lf, lb = new_group(pair), new_group(pair)
            if ctx.rank == pair[0]:
                ctx.link_f[1], ctx.link_b[1] = lf, lb
            elif ctx.rank == pair[1]:
                ctx.link_f[0], ctx.link_b[0] = lf, lb
        if multi and ctx.pp_virtual > 1:
            pair = [ranks[0], ranks[-1]]
            wf, wb = new_group(pair), new_group(pair)
            if ctx.rank in pair:
                ctx.wrap_f, ctx.wrap_b = wf, wb
    for s in range(pp):
        ranks = list(range(s, world, pp))
        g = new_group(ranks) if dp > 1 and world > 1 else None
        if ctx.rank in ranks:
            ctx.dp_group, ctx.dp_ranks = g, ranks
    if ctx.dp_group is None and dp == 1 and world == 1:
        ctx.dp_ranks = [0]
    if not ctx.pp_ranks:
        ctx.pp_ranks = [ctx.rank]


def get() -> DistContext:
    if _CTX is None:
        return init(verbose=False, sanity=False)
    return _CTX


def is_initialized() -> bool:
    return _CTX is not None


def barrier():
    if dist.is_initialized():
        c = get()
        dist.barrier(group=c.ctrl_group)


def broadcast_obj(obj, src: int = 0):
    """Rank ``src``'s picklable ``obj`` on every rank (gloo control plane; identity when single).

    Used for run-wide choices that must not depend on a per-rank clock or environment
    (e.g. the run directory name: every rank must checkpoint into the same place)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=src, group=get().ctrl_group)
    return box[0]


def destroy():
    global _CTX
    if dist.is_initialized():
        try:
            dist.barrier()
        except Exception:
            pass
        dist.destroy_process_group()
    _CTX = None


def hostname():
    return socket.gethostname()
