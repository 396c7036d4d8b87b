"""Pipeline micro-batch planner: pick the micro-batch size of a PP run for 288 GB HBM.

The reference runs DeepSpeed's 1F1B with micro-batch 1 and 96 micro-batches per optimizer step
(`P2/submit_opt27b_pp.sbatch:26-32`); on MI355X that shape leaves the matrix cores
idle (a 512-row GEMM), while one huge micro-batch maximises the pipeline bubble.  For a fixed
per-replica batch B (sequences per optimizer step), S stages and micro-batch mb (m = B / mb
micro-batches):

    step(mb) ≈ (m + S − 1) · T_stage(mb) + 2 (S − 1) · hop(mb)
    T_stage(mb) = max over stages of  layers_s · c_layer(mb·seq) · mb·seq  (+ embed / head work)
    hop(mb)     = mb·seq·d·bytes / link_bw + link_latency

``c_layer(T)`` is the measured per-token cost of one decoder layer's forward + backward at a
micro-batch of T tokens on one GPU (``tools/mb_sweep.py``, dp1, graph-replayed steps), kept per
model in ``MEASURED``; between samples it is interpolated in log(T), outside them the
``c_inf · (1 + T0 / T)`` fit is used.  The memory bound: stage s keeps up to S − s micro-batches
of saved activations alive (1F1B), so stage 0 needs S · mb · seq · act_bytes_per_token · layers_0
on top of its weights; candidates that do not fit ``hbm_budget`` are dropped.

``choose_micro_batch`` returns the fastest feasible mb together with the prediction, including
the per-GPU efficiency against the best dp1 micro-batch (one GPU, no bubble), so a run records
WHY it used the micro-batch it used.

Interleaved 1F1B (``virtual`` V model chunks per rank, parallel/pipeline.py) cuts the bubble term
to (S − 1)/V stage-times: step(mb, V) ≈ (m + (S − 1)/V) · T_stage(mb) + 2 (S·V − 1)/S · hop(mb)
(every micro-batch now crosses S·V − 1 stage boundaries, spread over S ranks).  It needs
m % S == 0 and S·V ≤ layers; ``choose_micro_batch(..., virtual="auto")`` searches (mb, V) jointly.
The memory bound grows with the deeper warm-up: rank 0 keeps up to 2(S − 1) + (V − 1)·S + 1
chunk-micro-batches of L/(S·V) layers alive.
"""
import math

GiB = 1 << 30

# ms per sequence of a whole dp1 optimizer step (all layers + embed + head + optimizer), seq 512,
# 96 sequences per step, fp16, fused HIP path, graph replay: tools/mb_sweep.py on one MI355X
# (profiles/r4/mb_sweep_opt67b.jsonl; OPT-2.7B mb >= 4 re-measured after the round-4 kernel hygiene —
# in-kernel pad-id ignore and loss sum, two-launch optimizer, in-launch lora_proj reduction:
# profiles/r4/mb_sweep_opt27b_r4k.jsonl; mb 1, 2 from the first sweep, mb_sweep_opt27b.jsonl).
MEASURED = {
    "opt-2.7b": {1: 25.5406, 2: 14.4509, 4: 11.5326, 8: 7.9711, 12: 6.7671, 16: 7.3182, 24: 6.4964, 48: 6.3744},
    "opt-6.7b": {1: 34.2091, 2: 20.8388, 4: 18.9054, 8: 14.9082, 16: 14.7781, 32: 14.7251},
}

LINK_BW = 100e9        # bytes/s one xGMI link achieves for a large RCCL p2p (≈153 GB/s raw)
LINK_LAT = 20e-6       # s per p2p message


def _norm(name):
    return name.lower().split("/")[-1]


def cost_per_seq_ms(model_name, mb, measured=None):
    """dp1 ms per sequence at micro-batch ``mb`` (interpolated in log(mb) between samples)."""
    tab = (measured or MEASURED).get(_norm(model_name))
    if not tab:
        tab = MEASURED["opt-2.7b"]
    xs = sorted(tab)
    if mb in tab:
        return tab[mb]
    if len(xs) >= 2 and xs[0] <= mb <= xs[-1]:
        for lo, hi in zip(xs, xs[1:]):
            if lo <= mb <= hi:
                f = (math.log(mb) - math.log(lo)) / (math.log(hi) - math.log(lo))
                return tab[lo] + f * (tab[hi] - tab[lo])
    # c(mb) = c_inf (1 + m0 / mb) through the two extreme samples
    a, b = xs[0], xs[-1]
    ca, cb = tab[a], tab[b]
    if a == b or ca <= cb:
        return tab[min(xs, key=lambda x: abs(x - mb))]
    den = cb / a - ca / b
    m0 = (ca - cb) / den if den > 0 else 0.0
    m0 = max(m0, 0.0)
    c_inf = cb / (1.0 + m0 / b)
    return c_inf * (1.0 + m0 / mb)


def _divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


GRAPH_OP_OVERHEAD_S = 20e-6   # per chunk-micro-batch (fwd + bwd) when the stage graphs replay
EAGER_OP_OVERHEAD_S = 60e-6   # ... when the schedule runs eagerly (host-issued launches)


def stage_graphs_expected(recompute=False, fused=True):
    """Whether the PP engine will replay per-slot stage hipGraphs (the trainer's
    ``_fused_graphable("pipeline")``: fused GPU LoRA path, no recompute, MIFT_GRAPH not off)."""
    import os
    mode = os.environ.get("MIFT_GRAPH", "auto")
    return bool(fused) and not recompute and mode not in ("off", "0", "false", "")


def predict(cfg, seq, per_replica, stages, mb, split=None, measured=None, dtype_bytes=2, name=None, virtual=1,
            op_overhead_s=None, graphed=True, partition="balanced"):
    """Predicted step time and per-GPU efficiency of an S-stage pipeline at micro-batch ``mb``
    (``virtual`` > 1: interleaved schedule with that many model chunks per rank).

    Work is counted in layer-equivalents: a decoder layer is 1, the LM head V/(12 d) (on the last
    virtual stage), the partition is ``partition_layers(..., "balanced")`` over S·V virtual stages
    (or ``split``).  With u(mb) = dp1 time per layer-equivalent per micro-batch:
        step ≈ m·max_rank_units·u + (S − 1)·max_chunk_units·u + m·V·op_overhead + hops
    (the steady state runs at the slowest rank; warm-up and cool-down traverse the pipeline one
    chunk at a time).  ``partition``: "balanced" (whole layers) or "halves" (half-layer units).  ``op_overhead``: fixed cost per chunk-micro-batch (fwd + bwd): p2p latency and
    host launches — 20 µs graph-replayed (both schedules replay per-slot stage graphs since round 5),
    60 µs eager."""
    from .pipeline import attn_cost_fraction, partition_layers, split_chunk_costs
    name = name or getattr(cfg, "name_or_path", None) or "opt-2.7b"
    L = cfg.num_layers() if hasattr(cfg, "num_layers") else cfg.num_hidden_layers
    d = getattr(cfg, "hidden_size", None) or getattr(cfg, "n_embd")
    m = per_replica // mb
    v = max(1, int(virtual))
    nvs = stages * v
    head_layers = cfg.vocab_size / (12.0 * d)
    if split is None:
        split = partition_layers(L, nvs, partition, head_layers, ranks=stages, attn_frac=attn_cost_fraction(cfg))
    units = split_chunk_costs(split, head_layers, attn_frac=attn_cost_fraction(cfg))  # half-layer ends: sub-block
    rank_units = [sum(units[c * stages + r] for c in range(v)) for r in range(stages)]
    seq_ms = cost_per_seq_ms(name, mb, measured)          # whole model, dp1, per sequence
    u = seq_ms * 1e-3 * mb / (L + head_layers)             # s per layer-equivalent per micro-batch
    ovh = op_overhead_s if op_overhead_s is not None else (GRAPH_OP_OVERHEAD_S if graphed else EAGER_OP_OVERHEAD_S)
    hop = mb * seq * d * dtype_bytes / LINK_BW + LINK_LAT
    step = (m * max(rank_units) + (stages - 1) * max(units)) * u + m * v * ovh + 2 * (nvs - 1) / stages * hop
    best_dp1 = min(cost_per_seq_ms(name, x, measured) for x in _divisors(per_replica))
    dp1_step_per_gpu = best_dp1 * 1e-3 * per_replica / stages   # same work on S GPUs without a bubble
    return {"micro_batch": mb, "micro_batches": m, "virtual": v, "split": list(split), "op_overhead_us": ovh * 1e6,
            "stage_ms": round(max(rank_units) * u * 1e3, 3), "hop_ms": round(hop * 1e3, 4),
            "step_ms": round(step * 1e3, 2), "bubble": round((stages - 1) / (v * m + stages - 1), 4),
            "efficiency_vs_dp1": round(dp1_step_per_gpu / step, 4)}


def act_bytes_per_token_layer(cfg, dtype_bytes=2):
    """Saved activations of one decoder layer per token (fused path, no recompute): LN outputs,
    q/k/v/attention output, the FFN pre-activation and post-activation, residuals, LoRA T
    operands — about 16·d + 2·ffn elements."""
    d = getattr(cfg, "hidden_size", None) or getattr(cfg, "n_embd")
    ffn = getattr(cfg, "ffn_dim", None) or 4 * d
    return (16 * d + 2 * ffn) * dtype_bytes


def graph_slots(stages, micro_batches, virtual, rank=0):
    """Chunk-micro-batches of saved activations one captured stage-graph set holds on ``rank``: the
    per-slot graphs of parallel/pipeline.py (K = S − s + 1 slots for 1F1B, Σ_c K_c for the
    interleaved schedule), each keeping one forward's activations in its private pool."""
    if virtual <= 1:
        return stages - rank + 1
    from .pipeline import chunk_slot_counts
    return sum(chunk_slot_counts(stages, rank, micro_batches, virtual))


def choose_micro_batch(cfg, seq, per_replica, stages, dtype_bytes=2, hbm_bytes=288 * 10 ** 9,
                       hbm_frac=0.85, measured=None, name=None, candidates=None, virtual=1, graph_sets=None,
                       graphed=None, partition="balanced"):
    """The feasible micro-batch (divisor of ``per_replica``) with the shortest predicted step.
    ``virtual``: model chunks per rank (int), or "auto" to choose among 1, 2, 4, ... as well.
    Memory: rank 0's live activations at the end of the eager warm-up, or ``graph_sets`` captured
    slot sets of stage graphs (``MIFT_PP_GRAPH_SETS``, default 2: the epoch's ragged last step keeps
    its own set), whichever is larger (the eager step's cached blocks are released before a capture)."""
    import os
    if graphed is None:
        graphed = stage_graphs_expected()
    if graph_sets is None:
        graph_sets = int(os.environ.get("MIFT_PP_GRAPH_SETS", "2"))
    L = cfg.num_layers() if hasattr(cfg, "num_layers") else cfg.num_hidden_layers
    n_params = getattr(cfg, "num_params", None)
    d = getattr(cfg, "hidden_size", None) or getattr(cfg, "n_embd")
    ffn = getattr(cfg, "ffn_dim", None) or 4 * d
    layer_params = 4 * d * d + 2 * d * ffn
    weights = (layer_params * L / stages + cfg.vocab_size * d) * dtype_bytes
    budget = hbm_bytes * hbm_frac - weights
    if virtual == "auto":
        vs = [v for v in (1, 2, 4) if stages > 1 and 2 * stages * v <= L] or [1]  # >= 2 layers per chunk
    else:
        vs = [int(virtual)]
    best, table = None, []
    for v in vs:
        per_tok = act_bytes_per_token_layer(cfg, dtype_bytes) * math.ceil(L / (stages * v))
        for mb in candidates or _divisors(per_replica):
            m = per_replica // mb
            if v > 1 and m % stages:
                continue
            inflight = stages if v == 1 else min(2 * (stages - 1) + (v - 1) * stages + 1, m * v)
            held = max(inflight, graph_sets * graph_slots(stages, m, v)) if stages > 1 else inflight
            need = held * mb * seq * per_tok      # rank 0's live activations (eager warm-up or graph slots)
            p = predict(cfg, seq, per_replica, stages, mb, measured=measured, dtype_bytes=dtype_bytes, name=name,
                        virtual=v, graphed=graphed, partition=partition)
            p["act_gib"] = round(need / GiB, 2)
            p["graph_slot_sets"] = graph_sets
            p["fits"] = need <= budget
            table.append(p)
            if p["fits"] and (best is None or p["step_ms"] < best["step_ms"] - 1e-9):
                best = p
    if not table:
        if vs != [1]:  # every (mb, V > 1) pair was excluded by the m % stages rule: plain 1F1B instead
            return choose_micro_batch(cfg, seq, per_replica, stages, dtype_bytes, hbm_bytes, hbm_frac, measured,
                                      name, candidates, 1, graph_sets, graphed, partition)
        raise ValueError(f"choose_micro_batch: no micro-batch candidate for per_replica={per_replica}, "
                         f"stages={stages}, virtual={virtual}")
    if best is None:
        best = table[0]
    out = dict(best)
    out["candidates"] = [{k: t[k] for k in ("micro_batch", "virtual", "step_ms", "efficiency_vs_dp1", "fits")}
                         for t in table]
    out["model"] = ("step = (m*max_rank + (S-1)*max_chunk)*u(mb) + m*V*overhead + hops; u(mb) from the dp1 "
                    "micro-batch sweep (profiles/r4/mb_sweep_*.jsonl)")
    del n_params
    return out
