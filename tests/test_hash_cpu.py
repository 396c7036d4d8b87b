"""The torch re-implementation of the kernel dropout hash matches a numpy uint64 model."""
import numpy as np
import torch

from mift.ops import reference as ref


def _np_hash(seed, idx):
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return ((z ^ (z >> np.uint64(31))) >> np.uint64(32)).astype(np.int64)


def test_hash_matches_numpy():
    idx = np.arange(0, 100000, 7, dtype=np.int64)
    for seed in (0, 1, 123456789, (1 << 63) + 5):
        a = ref.mift_hash(seed, torch.from_numpy(idx)).numpy()
        b = _np_hash(seed, idx)
        assert (a == b).all()


def test_keep_rate():
    m = ref.keep_mask(42, (1000, 100), 0.1)
    rate = m.float().mean().item()
    assert abs(rate - 0.9) < 0.01
