"""Drop-in for the reference's ``utils/parallel_utils.py``: same three helpers,
backed by mift's bring-up (RCCL over xGMI on MI355X, gloo on CPU, SLURM env fallbacks).

``init_distributed(local_rank)`` keeps the reference contract: WORLD_SIZE>1 -> GPU backend
(``nccl`` = RCCL on ROCm) when GPUs exist else gloo, binding ``local_rank`` to its GPU;
WORLD_SIZE==1 still forms a one-rank gloo group so single-process runs take the same path.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch.distributed as dist  # noqa: E402

from mift.parallel import dist as _D  # noqa: E402


def init_distributed(local_rank: int = 0) -> None:
    os.environ.setdefault("LOCAL_RANK", str(local_rank))
    world = int(os.environ.get("WORLD_SIZE", os.environ.get("SLURM_NTASKS", "1")))
    backend = None if world > 1 else "gloo"
    _D.init(backend=backend, sanity=False, verbose=False)


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def is_main_process() -> bool:
    return (not dist.is_initialized()) or dist.get_rank() == 0
