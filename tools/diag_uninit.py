"""Uninitialised-memory probe: torch.empty* (and at::empty in the extension) return NaN-filled
memory under deterministic mode, so any kernel that reads memory it never wrote shows up as a
NaN loss / parameter.  Runs the eager fused training step of the graph test."""
import sys
import torch
sys.path.insert(0, ".")
torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
from tests.test_graph_gpu import _run

name = sys.argv[1] if len(sys.argv) > 1 else "distilgpt2"
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
graph = len(sys.argv) > 3 and sys.argv[3] == "graph"
le, pe, tr = _run(graph, name, precision=prec)
print("losses", le)
print("param finite", bool(torch.isfinite(pe).all()), "grad finite", bool(torch.isfinite(tr.arena.grad).all()))
