"""verify_replicas (parallel/ddp.py): exact at construction; the periodic check tolerates and heals an
ulp-level drift (a one-shot all-reduce may sum in a rank-dependent order) but raises on divergence."""
import pytest
import torch

from mift.utils import harness


def _w(rank, world, delta, rtol):
    import torch.distributed as dist
    from mift.parallel import dist as D
    from mift.parallel.ddp import verify_replicas
    D.init(verbose=False, sanity=False)
    t = torch.linspace(-1.0, 1.0, 1000)
    if rank == 1:
        t[17] += delta
    try:
        ok = verify_replicas([t], rtol=rtol, resync=True)
        err = None
    except RuntimeError as e:
        ok, err = None, str(e)
    # after a resync every rank holds rank 0's tensor
    same = verify_replicas([t]) if err is None else None
    D.destroy()
    return {"ok": ok, "err": err, "same": same}


def test_exact_replicas_pass():
    r = harness.run(_w, 2, timeout=120, delta=0.0, rtol=0.0)
    assert all(x["ok"] is True for x in r)


def test_any_difference_raises_without_tolerance():
    r = harness.run(_w, 2, timeout=120, delta=1e-7, rtol=0.0)
    assert all(x["err"] and "divergence" in x["err"] for x in r)


def test_ulp_drift_is_tolerated_and_resynced():
    r = harness.run(_w, 2, timeout=120, delta=1e-7, rtol=1e-5)
    assert all(x["ok"] is False and x["err"] is None and x["same"] is True for x in r)


@pytest.mark.parametrize("delta", [1e-3, 5.0])
def test_real_divergence_raises_with_tolerance(delta):
    r = harness.run(_w, 2, timeout=120, delta=delta, rtol=1e-5)
    assert all(x["err"] and "spread" in x["err"] for x in r)


def _w_slices(rank, world):
    from mift.parallel import dist as D
    from mift.parallel.ddp import verify_replicas
    D.init(verbose=False, sanity=False)
    big = torch.linspace(-1.0, 1.0, 1000)
    small = torch.full((100,), 1e-6)          # e.g. LoRA B early in training
    t = torch.cat([big, small])
    m = torch.zeros(1100)
    if rank == 1:
        t[1050] += 1e-6    # 100 % of the small slice's scale, 1e-6 of the arena's
        m[5] = 1.0
    out = {}
    for name, sl in [("whole", None), ("sliced", [[(0, 1000), (1000, 100)]])]:
        try:
            verify_replicas([t.clone()], rtol=1e-5, resync=False, slices=sl)
            out[name] = None
        except RuntimeError as e:
            out[name] = str(e)
    t2 = torch.linspace(-1.0, 1.0, 1000)
    if rank == 1:
        t2[3] += 1e-7
    verify_replicas([t2], rtol=1e-5, resync=True, companions=[[m]])
    out["m_synced"] = float(m[5])
    D.destroy()
    return out


def test_spread_is_judged_per_parameter_slice():
    """A real divergence inside a small-magnitude slice passes the arena-wide scale but not the per-slice
    one; a resync also re-broadcasts the companion optimizer state."""
    r = harness.run(_w_slices, 2, timeout=120)
    for x in r:
        assert x["whole"] is None
        assert x["sliced"] and "slice [1000, 1100)" in x["sliced"]
        assert x["m_synced"] == 0.0
