"""Minimal repro for rocprofv3 --pmc on hipGraph replays: capture N tiny kernels
(in-place adds on one small tensor) into one torch CUDA graph and replay it R times.  Run under
``rocprofv3 --pmc SQ_WAVES -- python3 tools/diag_pmc_graph.py N`` with and without
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0.  Prints the result check (every add applied once per replay)."""
import sys

import torch


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    x = torch.zeros(1024, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            x.add_(1.0)
    x.zero_()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    ok = bool((x == float(n * reps)).all())
    print(f"graph of {n} kernels replayed {reps}x: {'ok' if ok else 'WRONG'} (x[0] = {float(x[0])})", flush=True)


if __name__ == "__main__":
    main()
