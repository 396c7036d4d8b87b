"""Does the LM-head dgrad pay for E's row stride?  The split-K dgrad reads, per chunk, a 6288-column
slice of E [8192, 50304] (row stride 100 KB).  Proxy: the same 768 tiles as one GEMM of 8 x 8192 rows
at K = 6272, with A contiguous (row stride 12.5 KB) vs A a column slice of a [65536, 50304] matrix
(row stride 100 KB), tiles 8 and 10, interleaved rounds in one process."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mift  # noqa: E402


def timeit(fn, iters=10, rounds=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters)
    return statistics.median(ts)


def main():
    import mift._C as C
    M, N, K, ld = 8 * 8192, 768, 6272, 50304
    dt = torch.bfloat16
    big = torch.randn(M, ld, device="cuda", dtype=dt)
    a_str = big[:, :K]
    a_con = a_str.contiguous()
    b = torch.randn(N, K, device="cuda", dtype=dt)
    g = lambda a, t: C.gemm_nt(a, b, None, None, None, 0, None, None, 0.0, 3, False, 1.0, None, t, None, None, 0.0, 7)[0]  # noqa: E731
    assert torch.equal(g(a_str, 8), g(a_con, 8))
    res = {}
    for _ in range(3):
        for t in (8, 10):
            for name, a in (("contig", a_con), ("stride100KB", a_str)):
                res.setdefault(f"t{t}_{name}", []).append(timeit(lambda: g(a, t)))
    print(json.dumps({k + "_us": round(min(v) * 1e3, 1) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
