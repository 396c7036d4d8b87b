"""The torch re-implementation of the kernel dropout hash matches a numpy uint32 model."""
import numpy as np
import torch

from mift.ops import reference as ref


def _mix(x):
    x = x ^ (x >> np.uint32(16))
    x = x * np.uint32(0x7FEB352D)
    x = x ^ (x >> np.uint32(15))
    x = x * np.uint32(0x846CA68B)
    return x ^ (x >> np.uint32(16))


def _np_bits16(seed, idx):
    with np.errstate(over="ignore"):
        pair = (idx >> 1).astype(np.uint64)
        lo = (pair & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = (pair >> np.uint64(32)).astype(np.uint32)
        s_lo, s_hi = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
        h = _mix((lo * np.uint32(0x9E3779B9)) ^ _mix(hi ^ s_hi) ^ s_lo)
        sh = ((idx & 1) * 16).astype(np.uint32)
        return ((h >> sh) & np.uint32(0xFFFF)).astype(np.int64)


def test_hash_matches_numpy():
    idx = np.concatenate([np.arange(0, 100000, 7, dtype=np.int64), np.array([2 ** 33 + 5, 2 ** 40 + 2])])
    for seed in (0, 1, 123456789, (1 << 63) + 5):
        a = ref.mift_bits16(seed, torch.from_numpy(idx)).numpy()
        b = _np_bits16(seed, idx)
        assert (a == b).all()


def test_keep_rate():
    m = ref.keep_mask(42, (1000, 100), 0.1)
    rate = m.float().mean().item()
    assert abs(rate - 0.9) < 0.01
