"""Diagnose graph-vs-eager drift: eager twice, graph twice; per-step losses and per-tensor param diffs."""
import sys
import torch
sys.path.insert(0, ".")
from tests.test_graph_gpu import _run

name = sys.argv[1] if len(sys.argv) > 1 else "distilgpt2"
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
le, pe, tr = _run(False, name, precision=prec)
le2, pe2, _ = _run(False, name, precision=prec)
lg, pg, trg = _run(True, name, precision=prec)
lg2, pg2, _ = _run(True, name, precision=prec)
print("eager ", le)
print("eager2", le2)
print("graph ", lg)
print("graph2", lg2)
print("noise eager", (pe - pe2).abs().max().item(), "graph-graph", (pg - pg2).abs().max().item(),
      "eager-graph", (pe - pg).abs().max().item())
arena = tr.arena
for (n, p), off in zip(arena.named, arena.offsets):
    o = off if isinstance(off, int) else off[0]
    de = (pe[o:o + p.numel()] - pg[o:o + p.numel()]).abs().max().item()
    dn = (pe[o:o + p.numel()] - pe2[o:o + p.numel()]).abs().max().item()
    if de > 2e-4 or dn > 2e-4:
        print(f"{n:60s} eager-graph {de:.3e} eager-eager {dn:.3e}")
d = (pe - pg).abs()
idx = torch.topk(d, 10).indices
print("top diffs idx", idx.tolist(), d[idx].tolist(), "pe", pe[idx].tolist(), "pg", pg[idx].tolist())
for nm, a, b in (("eager-eager", pe, pe2), ("eager-graph", pe, pg), ("graph-graph", pg, pg2)):
    dd = (a - b).abs()
    print(nm, "frac>2e-4", (dd > 2e-4).float().mean().item(), "max", dd.max().item())
