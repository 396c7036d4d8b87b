"""Persistent vs one-tile fused LM-head forward (MIFT_LM_PERSIST) and the tile raster (MIFT_GEMM_GROUP),
at the distilgpt2 and OPT-2.7B shapes: arms interleaved in one process (guide §5.4 rule 24), median of
5 rounds x 10 launches, random data; every arm's outputs compared bitwise with the one-tile kernel's."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mift.ops import kernels as K  # noqa: E402

ARMS = [("onetile", {"MIFT_LM_PERSIST": "0", "MIFT_LM_GROUP": "0"}),
        ("onetile_auto", {"MIFT_LM_PERSIST": "0"}),
        ("persist_g0", {"MIFT_LM_PERSIST": "1", "MIFT_LM_GROUP": "0"}),
        ("persist_auto", {"MIFT_LM_PERSIST": "1"}),
        ("persist_g4", {"MIFT_LM_PERSIST": "1", "MIFT_LM_GROUP": "4"}),
        ("persist_g8", {"MIFT_LM_PERSIST": "1", "MIFT_LM_GROUP": "8"}),
        ("persist_nostore", {"MIFT_LM_PERSIST": "1", "MIFT_LM_DBG": "1"})]


def setenv(env):
    for k in ("MIFT_LM_PERSIST", "MIFT_GEMM_GROUP", "MIFT_LM_GROUP", "MIFT_LM_DBG"):
        os.environ.pop(k, None)
    os.environ.update(env)


for name, M, d, V, dt in [("distilgpt2", 8192, 768, 50257, torch.bfloat16),
                          ("opt-2.7b.mb12", 6144, 2560, 50272, torch.float16)]:
    Vp = (V + 63) // 64 * 64
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, d, device="cuda", generator=g).to(dt)
    W = torch.zeros(Vp, d, device="cuda", dtype=dt)
    W[:V] = (0.05 * torch.randn(V, d, device="cuda", generator=g)).to(dt)
    lab = torch.randint(0, V, (M,), device="cuda", generator=g)
    outs = {}
    ts = {a: [] for a, _ in ARMS}
    for arm, env in ARMS:
        setenv(env)
        outs[arm] = [t.clone() for t in K.lmhead_fwd(x, W, lab, V)]
    for _ in range(5):
        for arm, env in ARMS:
            setenv(env)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                K.lmhead_fwd(x, W, lab, V)
            b.record()
            torch.cuda.synchronize()
            ts[arm].append(a.elapsed_time(b) * 100)
    setenv({})
    row = {"name": name, "M": M, "K": d, "V": V}
    for arm, _ in ARMS:
        row[arm + "_us"] = round(statistics.median(ts[arm]), 1)
        if arm != "onetile":
            ref = outs["onetile"]
            if arm == "persist_nostore":  # E not written: compare the statistics / loss only
                row[arm + "_same"] = all(torch.equal(p, q) for p, q in zip(outs[arm][1:], ref[1:]))
            else:
                row[arm + "_same"] = all(torch.equal(p, q) for p, q in zip(outs[arm], ref))
    fl = 2.0 * M * Vp * d
    row["persist_auto_tflops"] = round(fl / row["persist_auto_us"] / 1e6, 1)
    print(json.dumps(row), flush=True)
