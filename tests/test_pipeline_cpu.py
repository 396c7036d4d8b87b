"""Multi-process (gloo, CPU) coverage of the parallel engines.

Every configuration trains the same tiny OPT for 2 optimizer steps on the same
data and must reproduce the single-process run: DDP (dp2), pipeline (pp2,
with dropout ON — masks are counter-based so stages agree exactly), DP×PP
(dp2×pp2) and ZeRO-1 (dp2).  Also checks the 1F1B op order and the stage
partitioner (reference split rule `P2/finetune_lora_opt_pp.py:156-162`).
"""
import pytest
import torch

from mift.parallel.pipeline import partition_layers, schedule_1f1b
from mift.utils import harness


def _worker(rank, world, pp=1, zero=0, steps=2, mb=2, accum=4, dropout=0.0, partition="uniform",
            ckpt_dir=None, resume=None, p2p="link", virtual=1):
    import os
    os.environ["MIFT_PP_P2P"] = p2p
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.models.opt import OPTConfig
    from mift.parallel import dist as D
    from mift.parallel.pipeline import head_cost_layers, partition_layers, stage_chunks, stage_layer_range
    from mift.train.trainer import TrainConfig, Trainer

    ctx = D.init(pp=pp, verbose=False, sanity=True, virtual=virtual)
    cfg = OPTConfig.preset("opt-tiny")
    split = partition_layers(cfg.num_hidden_layers, ctx.pp * virtual, partition, head_cost_layers(cfg))
    lr_ = stage_layer_range(split, ctx.pp_rank) if virtual == 1 else stage_chunks(split, ctx.pp, virtual, ctx.pp_rank)
    model = build_causal_lm("opt-tiny", seed=3, layer_range=lr_, has_embed=ctx.is_first_stage,
                            has_head=ctx.is_last_stage)
    model.config.dropout = dropout
    L.inject(model, L.LoraConfig(r=4, lora_alpha=8, lora_dropout=0.05 if dropout else 0.0,
                                 target_modules=["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"]), seed=3)
    model.seed = 11
    ds = synthetic_openwebtext(64, 16, cfg.vocab_size, cfg.pad_token_id, seed=5, full_length=False, mean_tokens=10)
    batcher = MicroBatcher(ds, mb, accum, rank=ctx.dp_rank, world=ctx.dp)
    tc = TrainConfig(epochs=1, batch=mb, accum=accum, lr=1e-2, max_steps=steps, precision="fp32", logging_steps=1,
                     step_log="none", zero_stage=zero, save_steps=1 if ckpt_dir else 0, output_dir=ckpt_dir,
                     resume=resume)
    tr = Trainer(model, batcher, tc, ctx)
    hist = tr.train()
    state = tr.adapter_state()
    D.destroy()
    return {"loss": [h["loss"] for h in hist], "gn": [h["grad_norm"] for h in hist], "state": state,
            "split": split}


def _close_runs(a, b, tol=1e-4):
    assert len(a["loss"]) == len(b["loss"]) == 2
    for x, y in zip(a["loss"], b["loss"]):
        assert abs(x - y) <= tol * max(1.0, abs(y)), (a["loss"], b["loss"])
    for x, y in zip(a["gn"], b["gn"]):
        assert abs(x - y) <= 1e-3 * max(1.0, abs(y)), (a["gn"], b["gn"])
    assert a["state"].keys() == b["state"].keys() and len(a["state"]) == 4 * 6 * 2
    for k in a["state"]:
        torch.testing.assert_close(a["state"][k], b["state"][k], atol=2e-5, rtol=1e-4)


@pytest.fixture(scope="module")
def single():
    return harness.run(_worker, 1, accum=8)[0]


@pytest.fixture(scope="module")
def single_drop():
    return harness.run(_worker, 1, accum=4, dropout=0.1)[0]


def test_ddp_matches_single(single):
    r = harness.run(_worker, 2, accum=4)
    _close_runs(r[0], single)
    assert r[1]["state"] == {}


def test_pipeline_matches_single_with_dropout(single_drop):
    r = harness.run(_worker, 2, pp=2, accum=4, dropout=0.1)
    _close_runs(r[0], single_drop)


@pytest.mark.parametrize("p2p", ["shared", "blocking"])
def test_pipeline_p2p_modes(single_drop, p2p):
    """The round-2 replica-wide per-direction communicators and the blocking single-communicator
    fallback (MIFT_PP_P2P) train exactly like the default per-link layout."""
    r = harness.run(_worker, 2, pp=2, accum=4, dropout=0.1, p2p=p2p)
    _close_runs(r[0], single_drop)


def test_ring_slot_reuse_is_checked():
    """A receive ring slot may be handed out again only after the compute reading it was queued
    (release): on RCCL a receive is ordered only behind work queued before its post."""
    from mift.parallel.pipeline import _Ring
    ring = _Ring(2, torch.float32, torch.device("cpu"))
    a, sa = ring.get((2, 3))
    b, sb = ring.get((2, 3))
    with pytest.raises(RuntimeError, match="reused before"):
        ring.get((2, 3))  # slot of `a` not released yet
    ring.release(sa)
    c, sc = ring.get((2, 3))
    assert sc == sa and c.data_ptr() == a.data_ptr()
    ring.release(sb)
    ring.release(sc)


def test_pipeline_4_stages_balanced(single_drop):
    r = harness.run(_worker, 4, pp=4, accum=4, dropout=0.1, partition="balanced")
    assert r[0]["split"] == [1, 1, 1, 1]
    _close_runs(r[0], single_drop)


def test_pipeline_half_layer_stages_match_single(single_drop):
    """Half-layer partition units (``partition_layers(..., "halves")``): stage boundaries that split a
    decoder layer between its attention and MLP sub-blocks (2 stages: [2.5, 1.5] layers; 4 stages:
    [1.5, 1, 1, 0.5]) reproduce the single-process run with dropout on, and the adapters gathered from
    the stages are exactly the model's (each half layer holds only its own sub-block's adapters)."""
    r = harness.run(_worker, 2, pp=2, accum=4, dropout=0.1, partition="halves")
    assert r[0]["split"] == [2.5, 1.5]
    _close_runs(r[0], single_drop)
    r = harness.run(_worker, 4, pp=4, accum=4, dropout=0.1, partition="halves")
    assert r[0]["split"] == [1.5, 1.0, 1.0, 0.5]
    _close_runs(r[0], single_drop)


def test_interleaved_half_layer_chunks_match_single(single_drop):
    r = harness.run(_worker, 2, pp=2, dropout=0.1, virtual=2, partition="halves")
    assert any(x != int(x) for x in r[0]["split"]), r[0]["split"]
    _close_runs(r[0], single_drop)


def test_half_layer_partition_balances_opt_configs():
    """BASELINE configs 3 / 5: whole-layer units leave the slowest rank 1.07 / 1.21 of the mean
    (profiles/r5/stage_time_config{3,5}.json); half-layer units bring the cost model to <= 1.03 / 1.08."""
    from mift.models.opt import OPTConfig
    from mift.parallel.pipeline import attn_cost_fraction, head_cost_layers, split_rank_costs
    for name, S, V, whole, half in (("opt-2.7b", 4, 4, 1.07, 1.03), ("opt-6.7b", 8, 2, 1.21, 1.08)):
        cfg = OPTConfig.preset(name)
        h, n, af = head_cost_layers(cfg), cfg.num_hidden_layers, attn_cost_fraction(cfg)
        for method, bound in (("balanced", whole + 0.01), ("halves", half)):
            split = partition_layers(n, S * V, method, h, ranks=S, attn_frac=af)
            assert sum(split) == n and all(x > 0 and 2 * x == int(2 * x) for x in split)
            c = split_rank_costs(split, S, h, attn_frac=af)
            assert max(c) / (sum(c) / S) <= bound, (name, method, split, c)


def test_dp_x_pp_matches_single(single):
    r = harness.run(_worker, 4, pp=2, accum=4)
    _close_runs(r[0], single)


def test_zero1_matches_single(single):
    r = harness.run(_worker, 2, zero=1, accum=4)
    _close_runs(r[0], single)


@pytest.mark.parametrize("partition", ["uniform", "halves"])
def test_pp_checkpoint_resume(tmp_path, single_drop, partition):
    """Stop after step 1 (checkpoint), resume in a fresh 2-stage job -> same result as uninterrupted
    (also with a stage boundary inside a decoder layer)."""
    d = str(tmp_path / "ck")
    harness.run(_worker, 2, pp=2, accum=4, dropout=0.1, steps=1, ckpt_dir=d, partition=partition)
    r = harness.run(_worker, 2, pp=2, accum=4, dropout=0.1, steps=2, ckpt_dir=d, resume="auto", partition=partition)
    for k in single_drop["state"]:
        torch.testing.assert_close(r[0]["state"][k], single_drop["state"][k], atol=2e-5, rtol=1e-4)


def test_interleaved_pipeline_matches_single(single_drop):
    """Interleaved 1F1B (2 ranks x 2 model chunks = 4 virtual stages of one layer each, the wrap-around
    links carry chunk 0's activations from rank 1 back to chunk 1 on rank 0) reproduces the
    single-process run with dropout on; adapters gathered from both chunks of both ranks."""
    r = harness.run(_worker, 2, pp=2, dropout=0.1, virtual=2)
    _close_runs(r[0], single_drop)


def test_interleaved_dp_x_pp(single):
    """2 DP replicas x 2 interleaved pipeline ranks (V = 2) == single process."""
    r = harness.run(_worker, 4, pp=2, virtual=2)
    _close_runs(r[0], single)


def test_interleaved_schedule_is_deadlock_free():
    """Blocking receives + asynchronous sends (the engine's execution model) complete every
    interleaved schedule: every rank count, chunk count and micro-batch count tried."""
    from mift.parallel.pipeline import schedule_interleaved, simulate_schedule
    for S in (2, 3, 4, 8):
        for V in (1, 2, 4):
            for M in (S, 2 * S, 4 * S):
                assert simulate_schedule(S, M, V) == 2 * S * M * V, (S, M, V)
    # every rank runs each (chunk, micro-batch) forward and backward exactly once
    ops = schedule_interleaved(4, 1, 8, 2)
    assert sorted(o for o in ops if o[0] == "F") == sorted(("F", c, i) for c in range(2) for i in range(8))
    assert sorted(o for o in ops if o[0] == "B") == sorted(("B", c, i) for c in range(2) for i in range(8))
    with pytest.raises(ValueError):
        schedule_interleaved(4, 0, 6, 2)  # micro-batches must be a multiple of the stages


def test_1f1b_schedule_order():
    S, M = 4, 6
    for s in range(S):
        ops = schedule_1f1b(S, s, M)
        assert sorted(ops) == sorted([("F", i) for i in range(M)] + [("B", i) for i in range(M)])
        live, peak = 0, 0
        for kind, i in ops:
            live += 1 if kind == "F" else -1
            peak = max(peak, live)
            if kind == "B":
                assert ("F", i) in ops[:ops.index(("B", i))]
        assert peak == min(S - s, M)


def test_partition_rules():
    assert partition_layers(32, 4, "uniform") == [8, 8, 8, 8]
    assert partition_layers(32, 5, "uniform") == [7, 7, 6, 6, 6]      # reference N//S + (i < N%S)
    b = partition_layers(32, 4, "balanced", head_layers=1.6)
    assert sum(b) == 32 and b[-1] < 8 and max(b[:-1]) <= 9
    assert sum(partition_layers(32, 8, "balanced", head_layers=1.6)) == 32


def test_interleaved_blocking_p2p_mode(single_drop):
    """MIFT_PP_P2P=blocking with the interleaved schedule: receives posted just in time (no one-op
    prefetch — under blocking receives that prefetch deadlocks at S = 2, V = 2, M = 2)."""
    r = harness.run(_worker, 2, pp=2, dropout=0.1, virtual=2, p2p="blocking")
    _close_runs(r[0], single_drop)
    # M = 2 micro-batches per step: the case the prefetch deadlocked; same result as the default layout
    a = harness.run(_worker, 2, pp=2, dropout=0.1, virtual=2, p2p="blocking", accum=2, mb=4)
    b = harness.run(_worker, 2, pp=2, dropout=0.1, virtual=2, accum=2, mb=4)
    _close_runs(a[0], b[0])


def test_chunk_slot_counts_cover_in_flight_micro_batches():
    """Interleaved stage graphs: slot i % K_c of chunk c is free again (its backward queued) before
    micro-batch i + K_c's receive is posted, for both receive policies."""
    from mift.parallel.pipeline import chunk_slot_counts, schedule_interleaved
    for S, V, M in [(2, 2, 2), (2, 2, 4), (4, 2, 8), (4, 4, 24), (8, 2, 16), (3, 3, 6)]:
        for pre in (True, False):
            for s in range(S):
                K = chunk_slot_counts(S, s, M, V, prefetch=pre)
                ops = schedule_interleaved(S, s, M, V)
                owner = [dict() for _ in range(V)]
                for j, (op, c, i) in enumerate(ops):
                    for jj in ((j, j + 1) if pre else (j,)):
                        if jj < len(ops) and ops[jj][0] == "F":
                            cc, ii = ops[jj][1], ops[jj][2]
                            k = ii % K[cc]
                            assert owner[cc].get(k, ii) == ii, (S, V, M, s, cc, ii)
                            owner[cc][k] = ii
                    if op == "B":
                        assert owner[c].pop(i % K[c]) == i
                assert all(k <= M for k in K)


def test_partition_balanced_by_rank():
    """Rank-balanced split for the interleaved pipeline (ranks=): every chunk keeps >= 1 layer, the
    layers sum up, and the last rank (which carries the head) holds fewer layers than the others."""
    for L_, S, V, head in [(32, 4, 4, 1.6), (32, 4, 2, 1.6), (32, 8, 2, 1.2), (24, 4, 2, 3.0), (8, 2, 2, 0.4)]:
        split = partition_layers(L_, S * V, "balanced", head_layers=head, ranks=S)
        assert sum(split) == L_ and min(split) >= 1 and len(split) == S * V, split
        per_rank = [sum(split[c * S + r] for c in range(V)) for r in range(S)]
        if int(head + 0.5) >= 1:
            assert per_rank[-1] < max(per_rank[:-1]), (split, per_rank)
        assert max(per_rank) - min(per_rank[:-1]) <= 1, (split, per_rank)


def _groups_worker(rank, world, mode, virtual=1):
    import os
    os.environ["MIFT_PP_P2P"] = mode
    from mift.parallel import dist as D
    ctx = D.init(pp=world, verbose=False, sanity=False, virtual=virtual)
    out = {"n": ctx.n_groups, "shared": ctx.pp_fwd_group is not None, "link": ctx.link_f != [None, None]}
    D.destroy()
    return out


@pytest.mark.parametrize("mode,virtual,n", [("link", 1, 1 + 2 * 3), ("blocking", 1, 1 + 2 * 3), ("shared", 1, 3),
                                            ("link", 2, 1 + 2 * 3 + 2)])
def test_grid_creates_only_the_selected_p2p_groups(mode, virtual, n):
    """4 pipeline ranks: the pipe group, then per-link pairs (link / blocking) OR the two replica-wide
    communicators (shared), plus the wrap-around pair when interleaved — never both layouts."""
    r = harness.run(_groups_worker, 4, mode=mode, virtual=virtual)
    assert r[0]["n"] == n, r
    assert r[0]["shared"] == (mode == "shared") and r[0]["link"] == (mode != "shared")
