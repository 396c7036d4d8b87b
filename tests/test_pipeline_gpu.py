"""Pipeline engine on the GPU fused path, multi-process on ONE MI355X over gloo (the rehearsal
transport): per-slot stage hipGraphs (parallel/pipeline.py _StageGraphs) must reproduce the eager
1F1B schedule, which must reproduce the single-process run (same data, dropout on)."""
import pytest
import torch

from mift.utils import harness

pytestmark = pytest.mark.gpu

GPU_ENV = {"MIFT_DEVICE": "cuda", "MIFT_BACKEND": "gloo"}


def _worker(rank, world, pp=1, graph=False, steps=3, mb=2, accum=6, p2p="link", max_grad_norm=1.0,
            consistency_every=0, zero=0, virtual=1, partition="uniform"):
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
    model = build_causal_lm("opt-tiny", dtype=torch.float16, device=ctx.device, seed=3,
                            layer_range=lr_, has_embed=ctx.is_first_stage, has_head=ctx.is_last_stage)
    model.config.dropout = 0.1
    L.inject(model, L.LoraConfig(r=4, lora_alpha=8, lora_dropout=0.05,
                                 target_modules=["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"]), seed=3)
    model.seed = 11
    ds = synthetic_openwebtext(mb * accum * steps * ctx.dp, 64, cfg.vocab_size, cfg.pad_token_id, seed=5,
                               full_length=False, mean_tokens=40)
    batcher = MicroBatcher(ds, mb, accum, rank=ctx.dp_rank, world=ctx.dp)
    tc = TrainConfig(epochs=1, batch=mb, accum=accum, lr=1e-3, max_steps=steps, precision="fp16", logging_steps=1,
                     step_log="none", save_steps=0, graph="on" if graph else "off", max_grad_norm=max_grad_norm,
                     consistency_every=consistency_every, consistency_rtol=0.0, zero_stage=zero)
    tr = Trainer(model, batcher, tc, ctx)
    hist = tr.train()
    state = tr.adapter_state()
    stats = dict(tr.engine.stats) if tr.engine is not None else {}
    D.destroy()
    return {"loss": [h["loss"] for h in hist], "gn": [h["grad_norm"] for h in hist],
            "state": {k: v.float() for k, v in state.items()}, "stats": stats}


def _close(a, b, tol):
    assert len(a["loss"]) == len(b["loss"]) == 3
    for x, y in zip(a["loss"], b["loss"]):
        assert abs(x - y) <= tol * max(1.0, abs(y)), (a["loss"], b["loss"])
    # grad norms every step: a replay that produced inf/NaN grads shows as a skipped step (norm 0)
    for x, y in zip(a["gn"], b["gn"]):
        assert y > 0 and abs(x - y) <= 2e-2 * y, (a["gn"], b["gn"])
    assert a["state"].keys() == b["state"].keys() and a["state"]
    for k in a["state"]:
        d = (a["state"][k] - b["state"][k]).abs().max().item()
        assert d <= 5e-3, (k, d)


@pytest.fixture(scope="module")
def single():
    return harness.run(_worker, 1, env=GPU_ENV, timeout=240)[0]


@pytest.mark.parametrize("pp", [2, 4])
def test_pipeline_graphs_match_eager_and_single(single, pp):
    eager = harness.run(_worker, pp, env=GPU_ENV, timeout=240, pp=pp, graph=False)
    graph = harness.run(_worker, pp, env=GPU_ENV, timeout=240, pp=pp, graph=True)
    for r in range(pp):
        assert graph[r]["stats"]["replays"] > 0, graph[r]["stats"]  # steps 2-3 replay the stage graphs
        assert eager[r]["stats"]["replays"] == 0
    _close(eager[0], single, 2e-3)
    _close(graph[0], eager[0], 1e-3)


@pytest.mark.parametrize("pp,virtual", [(2, 1), (4, 1), (2, 2)])
def test_half_layer_stages_on_gpu(single, pp, virtual):
    """Half-layer pipeline boundaries on the fused kernels (a stage ending after a layer's attention
    sub-block hands the residual stream to the next one, which runs that layer's MLP sub-block without
    the fused out_proj dropout-backward handoff): eager == single, stage graphs == eager."""
    r = harness.run(_worker, pp, env=GPU_ENV, timeout=240, pp=pp, virtual=virtual, partition="halves")
    _close(r[0], single, 2e-3)
    g = harness.run(_worker, pp, env=GPU_ENV, timeout=240, pp=pp, virtual=virtual, partition="halves", graph=True)
    assert g[0]["stats"]["replays"] > 0
    _close(g[0], r[0], 1e-3)


def test_interleaved_pipeline_on_gpu(single):
    """Interleaved 1F1B on the fused GPU kernels: 2 ranks x 2 model chunks (4 virtual stages of one
    layer each; chunk 0's activations return from rank 1 to rank 0 over the wrap-around link), eager
    == the single-process run, and the per-(chunk, slot) stage graphs (steps 2-3 replay) == eager."""
    r = harness.run(_worker, 2, env=GPU_ENV, timeout=240, pp=2, virtual=2)
    _close(r[0], single, 2e-3)
    g = harness.run(_worker, 2, env=GPU_ENV, timeout=240, pp=2, virtual=2, graph=True)
    for k in range(2):
        assert g[k]["stats"]["replays"] > 0 and r[k]["stats"]["replays"] == 0, (g[k]["stats"], r[k]["stats"])
    _close(g[0], r[0], 1e-3)


def test_interleaved_graphs_blocking_p2p(single):
    """The interleaved graphs with MIFT_PP_P2P=blocking (just-in-time receives) == single."""
    g = harness.run(_worker, 2, env=GPU_ENV, timeout=240, pp=2, virtual=2, graph=True, p2p="blocking")
    assert g[0]["stats"]["replays"] > 0
    _close(g[0], single, 2e-3)


@pytest.mark.parametrize("p2p", ["shared", "blocking"])
def test_pipeline_p2p_fallback_modes(single, p2p):
    r = harness.run(_worker, 2, env=GPU_ENV, timeout=240, pp=2, graph=True, p2p=p2p)
    _close(r[0], single, 2e-3)


@pytest.mark.parametrize("graph", [False, True])
def test_ddp_replicas_bit_identical_with_clipping_active(graph):
    """DP2 on the fused GPU kernels with clipping forced active every step (max_grad_norm=1e-3):
    each replica derives its clip coefficient from the all-reduced grads with the deterministic
    grad_stats kernel, so the replicas stay bit-identical — consistency_every=1 runs the exact
    checksum (verify_replicas) after every optimizer step and raises on any divergence (VERDICT r2
    #2; with the round-2 float-atomic grad_stats the coefficients could differ by ulps)."""
    r = harness.run(_worker, 2, env=GPU_ENV, timeout=240, graph=graph, max_grad_norm=1e-3, consistency_every=1)
    assert r[0]["loss"] == r[1]["loss"]
    assert all(g > 1e-3 for g in r[0]["gn"])  # the clip was active


@pytest.mark.parametrize("graph", [False, True])
def test_zero1_matches_ddp_on_gpu(graph):
    """DP2 + ZeRO-1 (reduce-scatter of the grad arena, sharded fused AdamW, all-gather) on the fused
    GPU path, eager and with the setup-time warm-up + hipGraph capture (which once launched
    grad_stats on an optimizer attribute Zero1AdamW lacked: every GPU ZeRO-1 run crashed at Trainer
    construction), equals plain DP2."""
    ref = harness.run(_worker, 2, env=GPU_ENV, timeout=240, graph=graph)
    z = harness.run(_worker, 2, env=GPU_ENV, timeout=240, graph=graph, zero=1)
    _close(z[0], ref[0], 1e-3)  # rank 0 holds the adapter state of plain DDP
    assert z[1]["loss"] == z[0]["loss"]
