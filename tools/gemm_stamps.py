"""Where a 256x256 GEMM launch spends its time, per block (gemm_set_stamps: wave 0's s_memtime at
entry / main loop started / main loop done / C tile in LDS / exit, s_memrealtime at entry and exit).

  python tools/gemm_stamps.py [--tiles 8,10]

Prints per (shape, tile, C-store on/off): the median cycles of prologue, main loop, epilogue phase 1
(accumulators -> LDS), epilogue phase 2 (LDS -> global, with the operand epilogue), and the spread of
block start / end times over the launch (100 MHz real-time clock, in us).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mift  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="8,10")
    ap.add_argument("--shapes", default="opt", help="opt | dgpt (the K = 768 distilgpt2 block GEMMs, bf16)")
    ap.add_argument("--ext", action="store_true", help="also time each shape with a LoRA K-extension (a2/b2)")
    ap.add_argument("--bias", action="store_true", help="with --ext: the variants add a bias instead")
    a = ap.parse_args()
    import mift._C as C
    if a.shapes == "dgpt":
        shapes, dt = [(8192, 3072, 768), (8192, 2304, 768), (8192, 768, 3072), (8192, 768, 768)], torch.bfloat16
    else:
        shapes, dt = [(6144, 7680, 2560), (6144, 2560, 2560), (6144, 2560, 640)], torch.float16
    for M, N, K in shapes:
        x = torch.randn(M, K, device="cuda", dtype=dt)
        w = torch.randn(N, K, device="cuda", dtype=dt)
        nblk = ((M + 63) // 64) * ((N + 63) // 64)  # >= the block count of any tile
        bias = torch.randn(N, device="cuda", dtype=dt)
        a2 = torch.randn(M, 32, device="cuda", dtype=dt)
        b2 = torch.randn(N, 32, device="cuda", dtype=dt)
        for tile, ext in [(int(t), e) for t in a.tiles.split(",") for e in ((0, 1) if a.ext else (0,))]:
            for store in ((1,) if a.ext else (1, 0)):
                os.environ["MIFT_LM_DBG"] = "0" if store else "1"
                buf = torch.zeros(nblk * 8, dtype=torch.int64, device="cuda")
                C.gemm_set_stamps(buf)
                for _ in range(3):
                    if a.bias:
                        C.gemm_nt(x, w, bias if ext else None, None, None, 0, None, None, 0.0, 0, False, 1.0,
                                  None, tile, None, None, 0.0, 0)
                    else:
                        C.gemm_nt(x, w, None, a2 if ext else None, b2 if ext else None, 0, None, None, 0.0, 0, False,
                                  1.0, None, tile, None, None, 0.0, 0)
                torch.cuda.synchronize()
                C.gemm_set_stamps(None)
                s = [b for b in buf.view(nblk, 8).cpu().tolist() if b[0] != 0]  # launched blocks only
                med = lambda v: statistics.median(v)  # noqa: E731
                row = {"shape": f"{M}x{N}x{K}", "tile": tile, "ext": bool(ext), "c_store": bool(store), "blocks": len(s)}
                if tile == 10:
                    row["prologue_cyc"] = med([b[1] - b[0] for b in s])
                    row["loop_cyc"] = med([b[2] - b[1] for b in s])
                else:
                    row["prologue+loop_cyc"] = med([b[2] - b[0] for b in s])
                row["epi1_cyc"] = med([b[3] - b[2] for b in s])
                row["epi2_cyc"] = med([b[4] - b[3] for b in s])
                row["block_cyc"] = med([b[4] - b[0] for b in s])
                t0 = min(b[6] for b in s)
                starts = sorted((b[6] - t0) / 100.0 for b in s)
                ends = sorted((b[7] - t0) / 100.0 for b in s)
                row["start_us_p50_max"] = [round(starts[len(starts) // 2], 2), round(starts[-1], 2)]
                row["end_us_min_p50_max"] = [round(ends[0], 2), round(ends[len(ends) // 2], 2), round(ends[-1], 2)]
                print(json.dumps(row), flush=True)
    os.environ.pop("MIFT_LM_DBG", None)


if __name__ == "__main__":
    main()
