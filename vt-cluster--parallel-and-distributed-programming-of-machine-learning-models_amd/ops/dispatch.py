"""Device dispatch: HIP kernels for GPU tensors, torch reference for CPU.

`use_kernels(t)` is True when `t` lives on the GPU and the user did not opt
out with MIFT_KERNELS=0.  If kernels are wanted but the extension is not
importable we raise (never a silent eager fallback on a GPU box).
"""
import torch

from .. import _ext


def use_kernels(t: torch.Tensor) -> bool:
    if not t.is_cuda:
        return False
    if not _ext.kernels_enabled():
        return False
    _ext.require()
    return True


def C():
    return _ext.require()
