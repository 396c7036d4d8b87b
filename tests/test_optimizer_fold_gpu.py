"""Two-launch optimizer (csrc/kernels/adamw.hip opt_stats + opt_apply, VERDICT r3 hygiene #8) against
the four-launch form (grad_stats -> grad_stats_reduce -> opt_finalize -> adamw): the same bits for
p / m / v / state in both finalize placements (inside opt_stats when no all-reduce follows, inside
opt_apply after one), over clean, inf and nan steps and with dynamic loss scaling."""
import pytest
import torch

from mift.ops.dispatch import C

pytestmark = pytest.mark.gpu


def _four(K, p, g, m, v, state, stats, lr, fin, adam):
    K.grad_stats(g, stats)
    K.opt_finalize(stats, state, *fin)
    K.adamw(p, g, m, v, torch.tensor([lr], device="cuda"), state, *adam)


def _two(K, p, g, m, v, state, stats, ws, lr, fin, adam, fin_in_apply):
    K.opt_stats(g, stats, ws, state, not fin_in_apply, *fin)
    K.opt_apply(p, g, m, v, lr, state, stats, ws, fin_in_apply, *fin, *adam)


@pytest.mark.parametrize("fin_in_apply", [False, True])
@pytest.mark.parametrize("n", [4099, 3_000_001])
def test_two_launch_optimizer_bit_identical(fin_in_apply, n):
    K = C()
    torch.manual_seed(0)
    p0 = torch.randn(n, device="cuda")
    A = [p0.clone(), None, torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")]
    B = [p0.clone(), None, torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")]
    sa = torch.tensor([0.0, 64.0, 0.0, 1.0, 0.0, 0.0], device="cuda")
    sb = sa.clone()
    sta, stb = torch.zeros(2, device="cuda"), torch.zeros(2, device="cuda")
    from mift.ops.kernels import ARRIVE_INTS
    ws = torch.zeros(ARRIVE_INTS + 32, dtype=torch.int32, device="cuda")
    fin = (1.0, True, 2.0, 0.5, 2)
    adam = (0.9, 0.999, 1e-8, 0.01)
    for i, kind in enumerate(["ok", "ok", "inf", "ok", "nan", "ok", "ok", "ok"]):
        g = torch.randn(n, device="cuda") * 30.0
        if kind == "inf":
            g[n // 3] = float("inf")
        elif kind == "nan":
            g[-1] = float("nan")
        A[1], B[1] = g.clone(), g.clone()
        lr = 1e-3 * (1 + i)
        _four(K, A[0], A[1], A[2], A[3], sa, sta, lr, fin, adam)
        _two(K, B[0], B[1], B[2], B[3], sb, stb, ws, lr, fin, adam, fin_in_apply)
        for x, y in zip(A + [sa, sta], B + [sb, stb]):
            assert torch.equal(x.view(torch.int32), y.view(torch.int32)), (i, kind)
        assert int(ws.abs().sum()) == 0
    assert sb.tolist()[0] == 6.0  # 8 steps, 2 skipped
