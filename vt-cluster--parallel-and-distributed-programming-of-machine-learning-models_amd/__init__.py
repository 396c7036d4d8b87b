"""mift — MI355X-native distributed LoRA fine-tuning framework.

Capability parity target: the VT-Cluster course project (reference mounted at
/root/reference): distilgpt2 LoRA DDP (``Cluster/Project 1``), OPT-2.7B LoRA
pipeline parallel + ZeRO-1 (``Cluster/Project 2``), tiny-BERT DDP train/infer
labs (``labs/tiny``), greedy generation probe and CPU RAG (``labs/ragging``).

Design (MI355X-first, see docs/ARCHITECTURE.md):
  * one process per GPU, ``torch.distributed`` over RCCL (xGMI) for the hot
    path, Gloo for the control plane and the CPU plumbing configuration;
  * hand-written HIP/CDNA4 kernels (MFMA + LDS) in ``csrc/kernels`` compiled
    for gfx950 into the in-tree extension ``mift._C``;
  * flat LoRA parameter / gradient arenas so the optimizer and the DDP
    all-reduce are single launches over one contiguous buffer;
  * frozen base weights stored once per K-major layout (fwd and dgrad) —
    HBM3E is 288 GB per GPU, so we trade memory for MFMA-friendly layouts.

Subpackages: models, ops, parallel, lora, train, data, infer, obs, utils.
"""
__version__ = "0.1.0"

from . import _ext  # noqa: F401  (extension loader; never raises on CPU)


def kernels_available() -> bool:
    """True when the gfx950 extension ``_C`` imported successfully."""
    return _ext.available()
