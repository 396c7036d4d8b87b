"""Packed per-step inputs of a replayed step (mift.train.graph.GraphedStep._layout): every
micro-batch tensor, the micro-step counters and 1/tokens get disjoint, 256-B aligned ranges of ONE
buffer, and views built from the layout round-trip the original tensors (CPU, no capture)."""
import torch

from mift.train.graph import GraphedStep


def test_layout_disjoint_aligned_roundtrip():
    g = torch.Generator().manual_seed(0)
    mbs = []
    for _ in range(3):
        mbs.append({"input_ids": torch.randint(0, 50000, (4, 37), generator=g),
                    "attention_mask": torch.randint(0, 2, (4, 37), generator=g),
                    "labels": torch.randint(-100, 50000, (4, 37), generator=g)})
    items, steps_off, inv_off, total = GraphedStep._layout(None, mbs)
    spans = sorted((off, off + n) for _, _, off, n, _, _ in items)
    spans += [(steps_off, steps_off + 8 * len(mbs)), (inv_off, inv_off + 4)]
    spans.sort()
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 <= b0, (a0, a1, b0, b1)
    assert all(off % 256 == 0 for _, _, off, _, _, _ in items) and steps_off % 256 == 0 and inv_off % 256 == 0
    assert spans[-1][1] <= total
    buf = torch.zeros(total, dtype=torch.uint8)
    for i, k, off, n, dt, shp in items:
        buf[off:off + n].view(dt).view(shp).copy_(mbs[i][k])
    buf[steps_off:steps_off + 24].view(torch.int64).copy_(torch.arange(11, 14))
    buf[inv_off:inv_off + 4].view(torch.float32).fill_(0.125)
    for i, k, off, n, dt, shp in items:
        assert torch.equal(buf[off:off + n].view(dt).view(shp), mbs[i][k])
    assert buf[steps_off:steps_off + 24].view(torch.int64).tolist() == [11, 12, 13]
    assert buf[inv_off:inv_off + 4].view(torch.float32).item() == 0.125


def test_capture_invalidates_multi_adapter_pack():
    """OPT's q/k/v adapters share one K-extension cached on a ConcatLinear (not an nn.Module). A
    hipGraph capture taken right after an eager pass at the same arena version must rebuild that
    operand inside the graph, otherwise every replay reads the pre-update LoRA weights (round-3
    bug: graphed OPT drifted from eager from step 2).  CPU: only the cache bookkeeping is checked."""
    from mift import lora as L
    from mift.models import build_causal_lm
    from mift.ops.fused import MultiAdapterOps, invalidate_packs
    m = build_causal_lm("opt-tiny", dtype=torch.float32, seed=0)
    L.inject(m, L.LoraConfig(r=8, lora_alpha=16, target_modules=["q_proj", "k_proj", "v_proj"]))
    L.LoraArena(m)
    cat = m.model.decoder.layers[0].self_attn.qkv
    a = MultiAdapterOps(cat, torch.float32)
    b = MultiAdapterOps(cat, torch.float32)
    assert b.A32s is a.A32s  # same arena version, no capture in between: cached
    invalidate_packs(m)
    c = MultiAdapterOps(cat, torch.float32)
    assert c.A32s is not a.A32s and torch.equal(c.A32s, a.A32s)
