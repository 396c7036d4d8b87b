"""Native prefetching loader (csrc/runtime/loader.cpp) vs the Python MicroBatcher path."""
import numpy as np
import pytest
import torch

import mift
from mift.data import MicroBatcher, synthetic_openwebtext


def _collect(mb, native, epoch=0, start=0):
    out = []
    for step in mb.epoch(epoch, start_step=start):
        out.append([{k: v.clone() for k, v in m.items()} for m in step])
    return out


@pytest.mark.skipif(not mift._ext.available(), reason="extension not built")
@pytest.mark.parametrize("mode,shuffle,world,rank", [("strided", False, 1, 0), ("strided", True, 3, 2),
                                                     ("contiguous", False, 2, 1)])
def test_native_loader_matches_python(mode, shuffle, world, rank):
    ds = synthetic_openwebtext(101, 24, 1000, 7, seed=4, full_length=False, mean_tokens=12)
    ds.ids[5, 3] = 7  # a pad-id token inside a valid region -> label -100 (collator rule)
    kw = dict(micro_batch=4, accum=3, rank=rank, world=world, mode=mode, shuffle=shuffle, seed=9)
    py = MicroBatcher(ds, native=False, **kw)
    nat = MicroBatcher(ds, native=True, **kw)
    assert nat.native
    for ep, start in [(0, 0), (1, 2)]:
        a, b = _collect(py, False, ep, start), _collect(nat, True, ep, start)
        assert len(a) == len(b) and len(a) > 0
        for sa, sb in zip(a, b):
            assert len(sa) == len(sb)
            for ma, mb_ in zip(sa, sb):
                for k in ("input_ids", "attention_mask", "labels"):
                    assert torch.equal(ma[k], mb_[k]), k


@pytest.mark.skipif(not mift._ext.available(), reason="extension not built")
def test_native_loader_restart_and_bounds():
    ds = synthetic_openwebtext(10, 8, 100, 0, seed=1)
    L = mift._ext.require().TokenLoader(torch.from_numpy(ds.ids), torch.from_numpy(ds.lengths), 0, 4, 2, False)
    L.start(torch.arange(10), 0)
    assert L.next()[0].shape == (4, 8)
    L.start(torch.tensor([9, 8, 7]), 0)  # restart mid-epoch: the old worker is stopped
    item = L.next()
    assert torch.equal(item[0], torch.from_numpy(ds.ids[[9, 8, 7]].astype(np.int64)))
    assert L.next() == []
    with pytest.raises(RuntimeError):
        L.start(torch.tensor([10]), 0)
