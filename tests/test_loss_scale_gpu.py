"""fp16 dynamic loss scaling on the MI355X path (VERDICT r3 Next #5): the HIP optimizer kernels
(grad_stats -> opt_finalize -> adamw, csrc/kernels/adamw.hip) against the reference math, and an
overflow on ONE pipeline stage / DP replica / ZeRO-1 shard skipping the step on every rank of a
multi-process run on one GPU (gloo transport, fused path, hipGraph-replayed steps)."""
import pytest
import torch

from mift.train.optim import FusedAdamW
from mift.utils import harness
from test_loss_scale_cpu import check_skip_agreed, ls_worker

pytestmark = pytest.mark.gpu

GPU_ENV = {"MIFT_DEVICE": "cuda", "MIFT_BACKEND": "gloo"}


def _pair(n=4099):
    torch.manual_seed(0)
    p = torch.randn(n)
    cpu = FusedAdamW(p.clone(), torch.zeros(n), lr=1e-2, loss_scale="dynamic", init_scale=8.0, growth_interval=2)
    gpu = FusedAdamW(p.clone().cuda(), torch.zeros(n, device="cuda"), lr=1e-2, loss_scale="dynamic", init_scale=8.0,
                     growth_interval=2)
    assert gpu.kernels and not cpu.kernels
    return cpu, gpu


def test_kernels_overflow_backoff_growth_match_reference():
    cpu, gpu = _pair()
    seq = ["ok", "inf", "nan", "ok", "ok", "ok", "inf"]
    for i, kind in enumerate(seq):
        g = torch.randn(cpu.g.numel()) * 4.0
        if kind == "inf":
            g[17] = float("inf")
        elif kind == "nan":
            g[-1] = float("nan")  # the ragged tail element
        cpu.g.copy_(g)
        gpu.g.copy_(g)
        p0 = gpu.p.clone()
        cpu.step()
        gpu.step()
        sc, sg = cpu.stats(), gpu.stats()
        assert (sc["step"], sc["loss_scale"], sc["found_inf"]) == (sg["step"], sg["loss_scale"], sg["found_inf"]), \
            (i, sc, sg)
        if kind != "ok":
            assert torch.equal(p0, gpu.p), i  # skipped: bit-unchanged
        assert (gpu.g == 0).all()
        torch.testing.assert_close(gpu.p.cpu(), cpu.p, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(gpu.m.cpu(), cpu.m, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(gpu.v.cpu(), cpu.v, rtol=1e-5, atol=1e-9)
    # ok, inf (8->4), nan (->2), ok, ok (growth 2 -> 4), ok, inf (->2)
    assert gpu.stats()["loss_scale"] == 2.0 and gpu.stats()["step"] == 4


@pytest.mark.parametrize("pp,zero,fault", [(2, 0, "1:2:inf:grads"), (2, 0, "0:2:inf:grads"),
                                           (1, 0, "1:2:inf:grads"), (1, 1, "0:2:inf:grads")])
def test_overflow_on_one_rank_skips_every_rank(pp, zero, fault):
    res = harness.run(ls_worker, 2, env=GPU_ENV, timeout=240, pp=pp, zero=zero, fault=fault, device="cuda",
                      graph="auto")
    check_skip_agreed(res)
