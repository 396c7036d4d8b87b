"""Pipeline parallelism: layer partitioning + a 1F1B micro-batch engine over RCCL p2p.

Replaces the reference's DeepSpeed ``PipelineModule`` / ``PipelineEngine``
(`P2/finetune_lora_opt_pp.py:114-224`) with a
design that also fixes its defects:

  * stage-local construction: each rank builds ONLY its stage's weights
    (``build_causal_lm(..., layer_range=..., has_embed=..., has_head=...)``),
    the reference materialises the whole fp32 OPT-2.7B on every rank first
    and is OOM-killed;
  * the split is honoured exactly and recorded (the DS partitioner re-split
    the STAGES+2 items, B5); ``partition="uniform"`` reproduces the
    reference's ``N//S + (i < N%S)`` rule (`:156-162`), ``"balanced"`` also
    charges the LM head (V·d MACs ≈ V/(12·d) decoder layers) to the last
    stage — the default, because the head is 1.6 OPT-2.7B layers;
  * only hidden states travel between stages: every stage of a replica reads
    the SAME data micro-batches (sharded by DP rank, not global rank — B7),
    so masks / labels never cross the wire (the dict-passing of B3);
  * the schedule is non-interleaved 1F1B (DeepSpeed ``TrainSchedule``): warm-up
    ``S - s - 1`` forwards, steady one-forward-one-backward, cool-down; at most
    ``S - s`` micro-batches of activations are alive on stage s;
  * p2p ordering (the RCCL argument).  RCCL executes the p2p of ONE communicator in issue
    order on one stream, so a receive posted early blocks every later op of that communicator
    until its matching send arrives.  Each adjacent stage pair therefore gets TWO 2-rank
    communicators, one per direction (``ctx.link_f`` activations s -> s+1, ``ctx.link_b``
    gradients s+1 -> s; ``MIFT_PP_P2P=link``, default).  Every communicator then carries one
    message kind between one sender and one receiver, both in micro-batch order, so ops match
    FIFO and an early-posted receive can only wait for ITS send: stage s's "send y(i) to s+1"
    never queues behind its "recv x(i+1) from s-1" (round 2 put both on one replica-wide
    communicator per direction, coupling y(i) to the predecessor's next forward — VERDICT r2
    weak #6; kept as ``MIFT_PP_P2P=shared``).  ``MIFT_PP_P2P=blocking`` is the debugging fallback:
    one replica communicator, every receive posted just in time and completed before its
    consumer (no prefetch); sends stay asynchronous (blocking sends deadlock 1F1B: s blocked
    sending y(i) to s+1 while s+1 is blocked sending dX(j) to s).
    Deadlock freedom: receives are asynchronous and the compute stream waits on one only right
    before its consumer; the matching send precedes that consumer in the 1F1B dependency graph,
    which is acyclic.  RCCL makes a p2p's stream wait for the compute stream at POST time, so a
    receive buffer is safe to reuse once the compute that last read it has been queued — the
    rings below enforce exactly that order (``_Ring``: reuse of an unreleased slot raises);
  * hipGraph (GPU fused path, ``graph=True``): after one eager warm-up step per micro-batch
    shape, each stage captures one forward graph and one backward graph per ring slot (slot =
    micro-batch index mod (S - s + 1), the in-flight bound + the prefetched receive) and replays
    them; p2p stays outside the graphs.  A slot's static output (y, or dX for the previous
    stage) is rewritten by its next replay only after the compute stream waited for the send
    that read it.  OPT-2.7B at the reference's micro-batch issues ~250 launches per micro-batch
    from Python eagerly; a replay is one launch.

Interleaved 1F1B (``ctx.pp_virtual`` = V > 1, Narayanan et al. 2021 / Megatron-LM's
interleaved schedule): the layers are split into S·V virtual stages and rank s holds chunks
s, S + s, 2S + s, ... (``stage_chunks``), so a micro-batch visits every rank V times and the
bubble shrinks from (S−1)/(M+S−1) to (S−1)/(V·M+S−1) at the same micro-batch size — on MI355X
that is the lever: small micro-batches leave the matrix cores idle (tools/mb_sweep.py: OPT-2.7B
costs 1.7× per token at 4 sequences per micro-batch vs 48), so the pipeline wants FEW, LARGE
micro-batches, and the interleaving pays for the bubble that creates.  Activations of chunk c
leave the last rank for chunk c+1 on the first rank over a wrap-around pair of 2-rank
communicators (``ctx.wrap_f`` / ``ctx.wrap_b``); every communicator still carries one message
kind between one sender and one receiver in an order both agree on (the k-th forward of every
rank is the same (chunk, micro-batch), see ``schedule_interleaved``), receives are posted one op
ahead into fresh buffers and waited right before their consumer, sends are asynchronous — a
blocking-receive / async-send execution of this schedule is deadlock-free
(tests/test_pipeline_cpu.py simulates it for every rank count tried).  The interleaved path runs
eagerly (no stage graphs).

Loss normalisation: the last stage scales each micro-batch's summed token
loss by ``loss_scale / global_ntokens`` (token-count normalisation over the
whole optimizer step and all DP replicas), so PP, DP and single-GPU runs
produce the same update for the same data.
"""
import gc
import os
from collections import deque

import torch

from .comm import P2P


# The attention sub-block's share of an OPT decoder layer's forward + backward time, measured per hidden
# size (tools/half_layer_cost.py, fused path, LoRA on all six linears, seq 512: OPT-2.7B at micro-batch
# 12 1.321 / 1.441 ms, OPT-6.7B at 6 1.415 / 1.858 ms: profiles/r6/half_layer_cost.jsonl); other sizes
# interpolate; MIFT_PP_ATTN_FRAC overrides.
ATTN_FRACTION = {2560: 0.478, 4096: 0.432}


def attn_cost_fraction(cfg):
    e = os.environ.get("MIFT_PP_ATTN_FRAC")
    if e:
        return float(e)
    d = getattr(cfg, "hidden_size", None) or getattr(cfg, "n_embd", 2560)
    xs = sorted(ATTN_FRACTION)
    if d <= xs[0]:
        return ATTN_FRACTION[xs[0]]
    if d >= xs[-1]:
        return ATTN_FRACTION[xs[-1]]
    lo = max(x for x in xs if x <= d)
    hi = min(x for x in xs if x >= d)
    return ATTN_FRACTION[lo] if lo == hi else \
        ATTN_FRACTION[lo] + (d - lo) / (hi - lo) * (ATTN_FRACTION[hi] - ATTN_FRACTION[lo])


def partition_layers(n_layers, n_stages, method="uniform", head_layers=0.0, embed_layers=0.0, ranks=None,
                     attn_frac=None):
    """-> list of per-stage layer counts (sum = n_layers).

    ``ranks`` (interleaved pipeline, n_stages = ranks x chunks): "balanced" then balances the per-RANK
    sums (virtual stage k runs on rank k % ranks): equal chunks, the last chunk (which carries the
    head) shortened by the head's layer-equivalents, the removed layers spread over the other
    ranks' chunks from the front.

    "halves" (OPT): the partition unit is the half layer (attention sub-block, then MLP sub-block,
    costing ``attn_frac`` (``attn_cost_fraction(cfg)``) and 1 − attn_frac of a layer), counts are multiples of 0.5 and the per-rank
    costs (embedding on the first virtual stage, head on the last) are balanced: with whole layers
    OPT-6.7B's 32 layers + a ~1-layer head over 8 ranks leave one rank 5 layers against a 4.13 mean
    (slowest / mean 1.21, profiles/r5/stage_time_config5.json)."""
    if method == "halves":
        return _partition_halves(n_layers, n_stages, head_layers, embed_layers, ranks, attn_frac)
    if n_stages > n_layers:
        raise ValueError(f"{n_stages} stages > {n_layers} layers")
    if method == "uniform":
        return [n_layers // n_stages + (1 if i < n_layers % n_stages else 0) for i in range(n_stages)]
    if method == "balanced" and ranks and ranks > 1 and n_stages > ranks:
        split = [n_layers // n_stages + (1 if i < n_layers % n_stages else 0) for i in range(n_stages)]
        take = min(int(head_layers + 0.5), split[-1] - 1)
        split[-1] -= take
        k = 0
        while take > 0:  # round-robin over the chunks not on the last rank
            if k % ranks != ranks - 1:
                split[k] += 1
                take -= 1
            k = (k + 1) % (n_stages - 1)
        return split
    if method != "balanced":
        raise ValueError(method)
    # minimise the max stage cost; cost(stage) = layers + embed (first) + head (last)
    best = None
    lo = 0.0
    hi = n_layers + head_layers + embed_layers
    for _ in range(60):  # bisection on the bottleneck cost
        mid = (lo + hi) / 2
        split = _greedy(n_layers, n_stages, mid, head_layers, embed_layers)
        if split is not None:
            best, hi = split, mid
        else:
            lo = mid
    return best or partition_layers(n_layers, n_stages, "uniform")


def _greedy(n, S, cap, head, embed):
    split, left = [], n
    for s in range(S):
        extra = (embed if s == 0 else 0.0) + (head if s == S - 1 else 0.0)
        rem_stages = S - s - 1
        k = int(cap - extra + 1e-9)
        k = min(k, left - rem_stages)  # leave >= 1 layer per remaining stage
        if k < 1:
            return None
        if s == S - 1:
            if left > k:
                return None
            k = left
        split.append(k)
        left -= k
    return split if left == 0 else None


def _partition_halves(n_layers, n_stages, head, embed, ranks, attn_frac):
    if attn_frac is None:
        attn_frac = float(os.environ.get("MIFT_PP_ATTN_FRAC", 0.45))
    nu = 2 * n_layers
    if n_stages > nu:
        raise ValueError(f"{n_stages} stages > {nu} half layers")
    R = ranks if ranks and 1 < ranks < n_stages else n_stages
    cum = [0.0]
    for u in range(nu):
        cum.append(cum[-1] + (attn_frac if u % 2 == 0 else 1.0 - attn_frac))

    def rank_costs(b):
        c = [0.0] * R
        for k in range(n_stages):
            c[k % R] += cum[b[k + 1]] - cum[b[k]] + (embed if k == 0 else 0.0) + (head if k == n_stages - 1 else 0.0)
        return c

    def score(b):  # slowest rank first, then the spread
        c = rank_costs(b)
        return (round(max(c), 9), round(sum(x * x for x in c), 9))

    # boundaries at the cumulative cost targets (every virtual stage's share of the total, net of the
    # embedding / head it carries), then a local search
    total = cum[-1] + head + embed
    b, target = [0], 0.0
    for k in range(n_stages - 1):
        target += total / n_stages - (embed if k == 0 else 0.0)
        lo, hi = b[-1] + 1, nu - (n_stages - 1 - k)
        j = min(range(lo, hi + 1), key=lambda x: abs(cum[x] - target))
        b.append(j)
    b.append(nu)
    best = score(b)
    for _ in range(64):  # moves: shift any run of consecutive boundaries by one unit (converges in a few)
        improved = False
        for k1 in range(1, n_stages):
            for k2 in range(k1, n_stages):
                for dlt in (-1, 1):
                    if not (b[k1 - 1] < b[k1] + dlt and b[k2] + dlt < b[k2 + 1]):
                        continue
                    cand = b[:k1] + [x + dlt for x in b[k1:k2 + 1]] + b[k2 + 1:]
                    sc = score(cand)
                    if sc < best:
                        b, best, improved = cand, sc, True
        if not improved:
            break
    return [(b[k + 1] - b[k]) / 2 for k in range(n_stages)]


def split_chunk_costs(split, head=0.0, embed=0.0, attn_frac=None):
    """Cost (layer-equivalents) of every virtual stage of ``split``: its layers, a half layer at either
    end costed as its sub-block (``partition_layers(..., "halves")``), the embedding on the first and
    the head on the last."""
    if attn_frac is None:
        attn_frac = float(os.environ.get("MIFT_PP_ATTN_FRAC", 0.45))
    out, pos = [], 0.0
    for k, n in enumerate(split):
        lo, hi = pos, pos + n
        c = hi - lo
        if lo != int(lo):  # starts inside a layer: holds its MLP sub-block
            c += (1.0 - attn_frac) - 0.5
        if hi != int(hi):  # ends inside a layer: holds its attention sub-block
            c += attn_frac - 0.5
        out.append(c + (embed if k == 0 else 0.0) + (head if k == len(split) - 1 else 0.0))
        pos = hi
    return out


def split_rank_costs(split, ranks, head=0.0, embed=0.0, attn_frac=None):
    """Per-rank sums of ``split_chunk_costs`` (virtual stage k runs on rank k % ranks)."""
    costs = [0.0] * ranks
    for k, c in enumerate(split_chunk_costs(split, head, embed, attn_frac)):
        costs[k % ranks] += c
    return costs


def stage_layer_range(split, stage):
    lo = sum(split[:stage])
    return lo, lo + split[stage]


def stage_chunks(split, stages, virtual, stage):
    """Layer ranges held by pipeline rank ``stage`` when ``split`` partitions the layers over
    ``stages * virtual`` virtual stages: chunk c = virtual stage c·stages + stage."""
    if len(split) != stages * virtual:
        raise ValueError(f"split over {len(split)} virtual stages, expected {stages} x {virtual}")
    return [stage_layer_range(split, c * stages + stage) for c in range(virtual)]


def schedule_interleaved(S, s, M, V):
    """Op order of rank s in the interleaved 1F1B schedule: [('F' | 'B', chunk, micro-batch)].

    The k-th forward of EVERY rank is chunk (k mod S·V) // S of micro-batch (k // S·V)·S + k mod S;
    the k-th backward the same with the chunk order reversed.  Rank s runs
    min(2(S−s−1) + (V−1)·S, M·V) warm-up forwards (all of them when M == S), then one forward /
    one backward, then the remaining backwards.  Needs M % S == 0."""
    if V == 1:
        return [(op, 0, i) for op, i in schedule_1f1b(S, s, M)]
    if M % S:
        raise ValueError(f"interleaved schedule: {M} micro-batches is not a multiple of {S} stages")
    total = M * V

    def fwd(k):
        return (k % (S * V)) // S, (k // (S * V)) * S + k % S

    def bwd(k):
        c, i = fwd(k)
        return V - 1 - c, i

    nwarm = total if M == S else min(2 * (S - s - 1) + (V - 1) * S, total)
    ops = [("F",) + fwd(k) for k in range(nwarm)]
    for j in range(total - nwarm):
        ops.append(("F",) + fwd(nwarm + j))
        ops.append(("B",) + bwd(j))
    ops += [("B",) + bwd(k) for k in range(total - nwarm, total)]
    return ops


def simulate_schedule(S, M, V):
    """Execute every rank's op list with blocking receives and asynchronous sends; returns the
    number of ops run (== 2·S·M·V when the schedule cannot deadlock)."""
    ops = [schedule_interleaved(S, s, M, V) if V > 1 else [(o, 0, i) for o, i in schedule_1f1b(S, s, M)]
           for s in range(S)]
    done, pos, ran = set(), [0] * S, 0
    progress = True
    while progress:
        progress = False
        for s in range(S):
            while pos[s] < len(ops[s]):
                op, c, i = ops[s][pos[s]]
                vs = c * S + s
                if op == "F":
                    ok = vs == 0 or ("F", vs - 1, i) in done
                else:
                    ok = ("F", vs, i) in done and (vs == S * V - 1 or ("B", vs + 1, i) in done)
                if not ok:
                    break
                done.add((op, vs, i))
                pos[s] += 1
                ran += 1
                progress = True
    return ran


def head_cost_layers(cfg):
    """LM-head MACs in units of one decoder layer (12·d² MACs per token + attention ignored)."""
    d = getattr(cfg, "hidden_size", None) or getattr(cfg, "n_embd")
    ffn = getattr(cfg, "ffn_dim", None) or getattr(cfg, "n_inner", 4 * d)
    return cfg.vocab_size * d / (4 * d * d + 2 * d * ffn)


class PipelineEngine:
    """Runs one optimizer step's micro-batches through this rank's stage.

    ``model``: the stage model (``has_embed`` on stage 0, ``has_head`` on the
    last).  ``ctx``: mift.parallel.dist.DistContext (pp_rank, pp_ranks, ...)."""

    def __init__(self, model, ctx, act_dtype, hidden_size, graph=False):
        self.model, self.ctx = model, ctx
        self.S, self.s = ctx.pp, ctx.pp_rank
        self.first, self.last = self.s == 0, self.s == self.S - 1
        self.prev = ctx.pp_ranks[self.s - 1] if not self.first else None
        self.next = ctx.pp_ranks[self.s + 1] if not self.last else None
        self.mode = os.environ.get("MIFT_PP_P2P", "link")
        if self.mode in ("link", "blocking"):
            lf, lb = getattr(ctx, "link_f", [None, None]), getattr(ctx, "link_b", [None, None])
            self.rx_f, self.tx_f = P2P(lf[0]), P2P(lf[1])   # activations: from prev / to next
            self.rx_b, self.tx_b = P2P(lb[1]), P2P(lb[0])   # gradients: from next / to prev
        elif self.mode == "shared":
            f, b = P2P(getattr(ctx, "pp_fwd_group", None)), P2P(getattr(ctx, "pp_bwd_group", None))
            self.rx_f = self.tx_f = f
            self.rx_b = self.tx_b = b
        else:
            raise ValueError(f"MIFT_PP_P2P={self.mode!r}: link | shared | blocking")
        self.blocking = self.mode == "blocking"
        self.V = getattr(ctx, "pp_virtual", 1) or 1
        if self.V > 1:
            self.rx_wf, self.tx_wf = P2P(getattr(ctx, "wrap_f", None)), P2P(getattr(ctx, "wrap_f", None))
            self.rx_wb, self.tx_wb = P2P(getattr(ctx, "wrap_b", None)), P2P(getattr(ctx, "wrap_b", None))
            self.first_rank, self.last_rank = ctx.pp_ranks[0], ctx.pp_ranks[-1]
            if len(getattr(model, "chunk_ranges", [])) != self.V:
                raise ValueError(f"interleaved pipeline: the stage model holds "
                                 f"{len(getattr(model, 'chunk_ranges', []))} chunks, expected {self.V}")
        self.dtype, self.d = act_dtype, hidden_size
        self.device = ctx.device
        self.stats = {"fwd": 0, "bwd": 0, "replays": 0}
        # receive rings: an activation lives until its micro-batch's backward (at most S - s in
        # flight on stage s) plus the one prefetched ahead; a gradient only until its backward
        self.K = self.S - self.s + 1
        self._xring = _Ring(self.K, act_dtype, self.device, "activation")
        self._gring = _Ring(2, act_dtype, self.device, "gradient")
        self.graphs = _StageGraphs(self) if graph else None

    # ---- per-micro-batch compute ----
    def _act_shape(self, mb):
        b, S = mb["input_ids"].shape
        return (b, S, self.d)

    def _forward(self, mb, x, micro_step):
        m = self.model
        m.micro_step = micro_step
        emb, head = getattr(m, "embed_here", self.first), getattr(m, "head_here", self.last)  # chunk-aware
        out = m(input_ids=mb["input_ids"] if emb else None, attention_mask=mb["attention_mask"],
                labels=mb["labels"] if head else None, hidden_states=x, reduction="sum",
                return_logits=False)
        self.stats["fwd"] += 1
        return out["loss"].float() if head else out["hidden_states"]

    def _backward(self, y, x, grad_y, gscale):
        if self.last:
            (y * gscale).backward()
        else:
            torch.autograd.backward(y, grad_tensors=grad_y)
        self.stats["bwd"] += 1
        return x.grad if x is not None else None

    def _post(self, p2p, **kw):
        pend = p2p.post(**kw)
        if self.blocking and kw.get("recvs"):
            pend.wait()
        return pend

    # ---- schedule ----
    def train_batch(self, mbs, gscale, micro_step0):
        """1F1B over ``mbs`` (already on device).  Returns the summed loss (last stage) or None.

        micro-batch i runs with ``model.micro_step = micro_step0 + i`` on every
        stage, so dropout masks are identical to the non-pipelined run.

        Communication is asynchronous and posted AHEAD of the compute that needs it:
        the activation of micro-batch i+1 is requested before micro-batch i's forward runs,
        and the gradient for the next backward before the forward that precedes it, each
        into a reusable ring buffer.  On RCCL ``Pending.wait()`` only orders the compute
        stream behind the transfer, so the host never blocks and xGMI transfers overlap the
        forward / backward kernels."""
        if self.V > 1:
            run = self.graphs.runner(mbs, gscale, micro_step0) if self.graphs is not None else None
            return self._schedule_interleaved(mbs, run or _EagerChunkRun(self, mbs, gscale, micro_step0))
        if self.graphs is not None:
            run = self.graphs.runner(mbs, gscale, micro_step0)
            if run is not None:
                return self._schedule(mbs, run)
        return self._schedule(mbs, _EagerRun(self, mbs, gscale, micro_step0))

    # ---- interleaved 1F1B (V model chunks per rank) ----
    def _schedule_interleaved(self, mbs, run):
        """Rank s's op list of ``schedule_interleaved``.  Receives are posted one op ahead of their
        consumer (just in time under ``MIFT_PP_P2P=blocking``, whose ``_post`` waits on every receive:
        a prefetch there would block on op j+1's input before op j's output is sent — with S = 2,
        V = 2, M = 2 rank 0 would wait for the wrap-around activation of F(1, 0) before running F(0, 1),
        which rank 1 needs first: ADVICE r4).  ``run`` is the eager (``_EagerChunkRun``) or the
        replayed (``_ChunkGraphRun``) compute of one (chunk, micro-batch)."""
        S, s, V, M = self.S, self.s, self.V, len(mbs)
        ops = schedule_interleaved(S, s, M, V)
        nvs = S * V
        m = self.model
        posted, sends = {}, []
        pre = not self.blocking

        def vstage(c):
            return c * S + s

        def needs_recv(j):
            if j >= len(ops):
                return None
            op, c, i = ops[j]
            vs = vstage(c)
            if op == "F" and vs > 0:
                return op, c, i
            if op == "B" and vs < nvs - 1:
                return op, c, i
            return None

        def post(key):
            op, c, i = key
            if op == "F":  # activation of virtual stage vs - 1
                buf, slot = run.x_buffer(c, i)
                p2p, src = (self.rx_f, self.prev) if s > 0 else (self.rx_wf, self.last_rank)
            else:          # gradient from virtual stage vs + 1
                buf, slot = run.g_buffer(c, i)
                p2p, src = (self.rx_b, self.next) if s < S - 1 else (self.rx_wb, self.first_rank)
            posted[key] = (self._post(p2p, recvs=[(buf, src)]), slot)

        def take(key):
            if key not in posted:
                post(key)
            pend, slot = posted.pop(key)
            pend.wait()
            return slot

        try:
            for j, (op, c, i) in enumerate(ops):
                key = needs_recv(j)
                if key is not None and key not in posted:
                    post(key)
                if pre:
                    nxt = needs_recv(j + 1)  # one op of receive prefetch
                    if nxt is not None and nxt not in posted:
                        post(nxt)
                vs = vstage(c)
                m.active_chunk = c
                if op == "F":
                    xslot = take(("F", c, i)) if vs > 0 else None
                    y = run.forward(c, i, xslot)
                    if vs < nvs - 1:
                        p2p, dst = (self.tx_f, self.next) if s < S - 1 else (self.tx_wf, self.first_rank)
                        sends.append(run.send_y(c, i, self._post(p2p, sends=[(y.detach(), dst)])))
                else:
                    gslot = take(("B", c, i)) if vs < nvs - 1 else None
                    gx = run.backward(c, i, gslot)
                    if gslot is not None:
                        run.release_g(c, i, gslot)
                    if vs > 0:
                        p2p, dst = (self.tx_b, self.prev) if s > 0 else (self.tx_wb, self.last_rank)
                        sends.append(run.send_gx(c, i, self._post(p2p, sends=[(gx, dst)])))
                    run.release_x(c, i)
        finally:
            m.active_chunk = None
        for p in sends:
            if p is not None:
                p.wait()
        return run.finish()

    def _schedule(self, mbs, run):
        M = len(mbs)
        nwarm = min(self.S - self.s - 1, M)
        nsteady = M - nwarm
        live = deque()
        xq = deque()
        sends = []
        pre = not self.blocking  # prefetch receives ahead of the compute that needs them

        def post_x(i):
            if not self.first and i < M:
                buf, slot = run.x_buffer(i)
                xq.append((self._post(self.rx_f, recvs=[(buf, self.prev)]), slot))

        def take_x(i):
            if self.first:
                return None, None
            if not pre:
                post_x(i)
            pend, slot = xq.popleft()
            pend.wait()
            return run.x_input(i, slot), slot

        def post_g(b):
            if self.last:
                return None
            buf, slot = run.g_buffer(b)
            return self._post(self.rx_b, recvs=[(buf, self.next)]), slot

        def fwd(i, x):
            y = run.forward(i, x)
            if not self.last:
                sends.append(run.send_y(i, self._post(self.tx_f, sends=[(y.detach(), self.next)])))
            return y

        def bwd(b, gp):
            if gp is None and not pre:
                gp = post_g(b)
            bx, by, xslot = live.popleft()
            g = None
            if gp is not None:
                pend, gslot = gp
                pend.wait()
                g = run.g_input(b, gslot)
            gx = run.backward(b, by, bx, g)
            if gp is not None:
                run.release_g(gslot)
            if not self.first:
                sends.append(run.send_gx(b, self._post(self.tx_b, sends=[(gx, self.prev)])))
            run.release_x(b, bx, xslot)

        if pre:
            post_x(0)
        for i in range(nwarm):
            x, xs = take_x(i)
            if pre:
                post_x(i + 1)
            live.append((x, fwd(i, x), xs))
        for j in range(nsteady):
            i = nwarm + j
            gp = post_g(j) if pre else None  # grad of the oldest live micro-batch, requested before the forward
            x, xs = take_x(i)
            if pre:
                post_x(i + 1)
            live.append((x, fwd(i, x), xs))
            bwd(j, gp)
        for k in range(nwarm):
            b = nsteady + k
            bwd(b, post_g(b) if pre else None)
        for p in sends:
            if p is not None:
                p.wait()
        return run.finish()


class _EagerRun:
    """Eager per-micro-batch compute of one ``train_batch`` (autograd builds a fresh graph per
    micro-batch; receive buffers come from the engine's rings)."""

    def __init__(self, eng, mbs, gscale, micro_step0):
        self.e, self.mbs, self.gscale, self.ms0 = eng, mbs, gscale, micro_step0
        self.loss = torch.zeros((), dtype=torch.float32, device=eng.device) if eng.last else None

    def x_buffer(self, i):
        return self.e._xring.get(self.e._act_shape(self.mbs[i]))

    def x_input(self, i, slot):
        return self.e._xring.buf(slot).requires_grad_(True)

    def g_buffer(self, b):
        return self.e._gring.get(self.e._act_shape(self.mbs[b]))

    def g_input(self, b, slot):
        return self.e._gring.buf(slot)

    def forward(self, i, x):
        y = self.e._forward(self.mbs[i], x, self.ms0 + i)
        if self.e.last:
            self.loss.add_(y.detach())
        return y

    def backward(self, b, y, x, g):
        return self.e._backward(y, x, g, self.gscale)

    def send_y(self, i, pend):
        return pend

    def send_gx(self, b, pend):
        return pend

    def release_x(self, b, x, slot):
        if x is not None:
            x.grad = None  # the ring slot is reused by a later micro-batch
        if slot is not None:
            self.e._xring.release(slot)

    def release_g(self, slot):
        self.e._gring.release(slot)

    def finish(self):
        return self.loss


class _EagerChunkRun:
    """Eager compute of one interleaved ``train_batch``: a fresh receive buffer per message (the
    interleaved in-flight set has no ring bound to check), autograd graphs kept per (chunk, micro-batch)."""

    def __init__(self, eng, mbs, gscale, micro_step0):
        self.e, self.mbs, self.gscale, self.ms0 = eng, mbs, gscale, micro_step0
        self.nvs = eng.S * eng.V
        self.loss = torch.zeros((), dtype=torch.float32, device=eng.device) if eng.last else None
        self.live = {}

    def _last(self, c):
        return c * self.e.S + self.e.s == self.nvs - 1

    def x_buffer(self, c, i):
        buf = torch.empty(self.e._act_shape(self.mbs[i]), dtype=self.e.dtype, device=self.e.device)
        return buf, buf

    g_buffer = x_buffer

    def forward(self, c, i, x):
        if x is not None:
            x = x.requires_grad_(True)
        y = self.e._forward(self.mbs[i], x, self.ms0 + i)
        if self._last(c):
            self.loss.add_(y.detach())
        self.live[(c, i)] = (x, y)
        return y

    def backward(self, c, i, g):
        x, y = self.live.pop((c, i))
        if self._last(c):
            (y * self.gscale).backward()
        else:
            torch.autograd.backward(y, grad_tensors=g)
        self.e.stats["bwd"] += 1
        return x.grad if x is not None else None

    def send_y(self, c, i, pend):
        return pend

    send_gx = send_y

    def release_x(self, c, i):
        pass

    def release_g(self, c, i, slot):
        pass

    def finish(self):
        return self.loss


def chunk_slot_counts(S, s, M, V, prefetch=True):
    """Graph slots per model chunk on rank s of the interleaved schedule: the most micro-batches of
    chunk c in flight at once, from the post of the receive feeding F(c, i) (at the top of the op
    before it when receives are prefetched; F itself on the first virtual stage, which receives
    nothing) until B(c, i) has been queued.  Per chunk the forwards and the backwards both run in
    micro-batch order, so the in-flight set is a run of consecutive micro-batches and slot i % K_c is
    never handed to micro-batch i + K_c before B(c, i) — the condition RCCL needs for a receive into
    a reused buffer (``_Ring``)."""
    ops = schedule_interleaved(S, s, M, V)
    occ = [set() for _ in range(V)]
    K = [1] * V
    for j, (op, c, i) in enumerate(ops):
        for jj in ((j, j + 1) if prefetch else (j,)):
            if jj < len(ops) and ops[jj][0] == "F":
                occ[ops[jj][1]].add(ops[jj][2])
        for cc in range(V):
            if occ[cc]:
                assert max(occ[cc]) - min(occ[cc]) + 1 == len(occ[cc]), "in-flight set not consecutive"
            K[cc] = max(K[cc], len(occ[cc]))
        if op == "B":
            occ[c].discard(i)
    return K


class _Ring:
    """Receive buffers reused round-robin per shape (``n`` slots: the in-flight bound).

    ``get`` hands out the next slot and marks it busy; ``release`` is called once the compute
    that reads the slot has been QUEUED.  Reusing a busy slot raises: on RCCL the next receive
    into it would be ordered only behind work queued before its post."""

    def __init__(self, n, dtype, device, what="buffer"):
        self.n, self.dtype, self.device, self.what = max(1, n), dtype, device, what
        self.bufs, self.idx, self.busy = {}, {}, {}

    def get(self, shape):
        shape = tuple(shape)
        bufs = self.bufs.setdefault(shape, [])
        i = self.idx.get(shape, 0)
        slot = (shape, i % self.n)
        if self.busy.get(slot):
            raise RuntimeError(f"pipeline {self.what} ring slot {slot[1]} reused before the compute reading it "
                               f"was queued (ring of {self.n})")
        self.idx[shape] = i + 1
        if len(bufs) < self.n:
            bufs.append(torch.empty(shape, dtype=self.dtype, device=self.device))
        self.busy[slot] = True
        # a fresh leaf view per use: no autograd state (.grad, requires_grad) carries over
        return bufs[slot[1]].detach(), slot

    def buf(self, slot):
        return self.bufs[slot[0]][slot[1]].detach()

    def release(self, slot):
        self.busy[slot] = False


class _StageGraphs:
    """Per-slot forward / backward hipGraphs of one pipeline stage (see the module docstring).

    Slot k serves micro-batches i with i % K == k (K = S - s + 1).  Its static buffers: the
    micro-batch inputs, the received activation x_k (a leaf that requires grad), the micro-step
    counter read by every dropout kernel (csrc/common.h ``mift_seed``), the forward output y_k
    (held with its autograd graph: the saved activations stay allocated), the received gradient
    g_k and the backward output dX_k = x_k.grad.  Every slot has its OWN private memory pool: graphs
    that share a pool must replay in capture order (a block freed at the end of one capture is handed
    to the next), but 1F1B replays F(i+1) before B(i) — with one shared pool the backward of slot k
    overwrote slot k+1's saved activations (measured: NaN gradients from the first replayed step).
    Within a slot the order is the capture order (forward, then backward)."""

    def __init__(self, eng, max_sets=None):
        from collections import OrderedDict
        self.e = eng
        self.seen = set()
        # captured slot sets per micro-batch signature (LRU, bounded): an epoch whose last step has
        # a different shape replays its own set instead of evicting and recapturing the main one
        self.sets = OrderedDict()
        self.max_sets = max_sets or int(os.environ.get("MIFT_PP_GRAPH_SETS", "2"))
        self.gs = torch.zeros((), dtype=torch.float32, device=eng.device)

    @staticmethod
    def _signature(mbs):
        return tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(mbs[0].items())) + (len(mbs),)

    def runner(self, mbs, gscale, micro_step0):
        if any(self._signature([mb]) != self._signature([mbs[0]]) for mb in mbs):
            return None
        sig = self._signature(mbs)
        slots = self.sets.get(sig)
        if slots is None:
            if sig not in self.seen:
                self.seen.add(sig)
                return None  # eager warm-up step for this shape; capture on the next one
            while len(self.sets) >= self.max_sets:
                self.sets.popitem(last=False)  # least recently used signature
            slots = self._capture(mbs) if self.e.V == 1 else self._capture_chunks(mbs)
            self.sets[sig] = slots
        self.sets.move_to_end(sig)
        if self.e.V > 1:
            return _ChunkGraphRun(self, slots, mbs, gscale, micro_step0)
        return _GraphRun(self, slots, mbs, gscale, micro_step0)

    def _capture_slot(self, mbs, first, last, pack):
        """Forward + backward graphs of one slot (private pool).  ``first``: no received activation
        (the embedding runs here); ``last``: the loss head runs here (seeded by ``self.gs``);
        ``pack``: this capture rebuilds the per-step LoRA operand packs (the step's first replay)."""
        from ..ops import streams
        from ..ops.dispatch import C
        from ..ops.fused import invalidate_packs
        e = self.e
        sl = {"inp": {key: torch.empty_like(v) for key, v in mbs[0].items()},
              "step": torch.zeros(1, dtype=torch.int64, device=e.device),
              "send_y": None, "send_gx": None}
        for key, v in mbs[0].items():
            sl["inp"][key].copy_(v)
        if not first:
            sl["x"] = torch.zeros(e._act_shape(mbs[0]), dtype=e.dtype, device=e.device).requires_grad_(True)
        if not last:
            sl["g"] = torch.zeros(e._act_shape(mbs[0]), dtype=e.dtype, device=e.device)
        if pack:
            invalidate_packs(e.model)
        C().set_seed_step(sl["step"])
        gf, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        gc_was = gc.isenabled()
        gc.collect()
        gc.disable()  # no collection inside the captures (see train/graph.py)
        try:
            with torch.cuda.graph(gf, capture_error_mode="thread_local"):
                y = e._forward(sl["inp"], sl.get("x"), 0)
            with torch.cuda.graph(gb, pool=gf.pool(), capture_error_mode="thread_local"):
                if last:
                    (y * self.gs).backward(retain_graph=True)
                else:
                    torch.autograd.backward(y, grad_tensors=sl["g"], retain_graph=True)
                streams.join()
        finally:
            if gc_was:
                gc.enable()
        C().set_seed_step(None)
        sl.update(gf=gf, gb=gb, y=y, gx=(sl["x"].grad if not first else None))
        return sl

    def _captured(self, body):
        from ..models.layers import graph_seeds
        from ..ops import streams
        from ..ops.dispatch import C
        e = self.e
        torch.cuda.synchronize(e.device)
        gc.collect()
        torch.cuda.empty_cache()  # the eager warm-up's cached blocks: the slot pools are allocated next
        graph_seeds(True)
        streams.set_enabled(False)
        try:
            return body()
        finally:
            graph_seeds(False)
            streams.set_enabled(None)
            C().set_seed_step(None)
            e.stats["captures"] = e.stats.get("captures", 0) + 1
            torch.cuda.synchronize(e.device)

    def _capture(self, mbs):
        e = self.e

        def body():
            # the per-step LoRA operand pack is captured into slot 0's forward (the step's first replay)
            slots = [self._capture_slot(mbs, e.first, e.last, pack=(k == 0)) for k in range(e.K)]
            e.stats["fwd"] -= e.K  # the captures ran _forward once per slot (backward bypassed _backward)
            return slots

        return self._captured(body)

    def _capture_chunks(self, mbs):
        """Interleaved schedule: slots per (chunk, micro-batch mod K_c) (``chunk_slot_counts``), each
        with its own pool.  Every rank's first op is F(0, 0), so slot (0, 0)'s forward carries the LoRA
        operand packs; chunk c's multi-adapter packs are rebuilt inside its slot 0 (its first replay
        of every step), which the chunk's later slots then read."""
        e = self.e
        Ks = chunk_slot_counts(e.S, e.s, len(mbs), e.V, prefetch=not e.blocking)
        nvs = e.S * e.V

        def body():
            slots = []
            try:
                for c in range(e.V):
                    vs = c * e.S + e.s
                    e.model.active_chunk = c
                    slots.append([self._capture_slot(mbs, vs == 0, vs == nvs - 1, pack=(c == 0 and k == 0))
                                  for k in range(Ks[c])])
            finally:
                e.model.active_chunk = None
            e.stats["fwd"] -= sum(Ks)
            return slots

        return self._captured(body)


class _GraphRun:
    """Replay-based per-micro-batch compute of one ``train_batch`` (slot = i mod K)."""

    def __init__(self, gr, slots, mbs, gscale, micro_step0):
        self.gr, self.e, self.mbs, self.ms0 = gr, gr.e, mbs, micro_step0
        self.slots = slots
        self.K = gr.e.K
        gr.gs.copy_(gscale.reshape(()))
        self.steps = torch.arange(micro_step0, micro_step0 + len(mbs), dtype=torch.int64).to(
            self.e.device, non_blocking=True)
        self.loss = torch.zeros((), dtype=torch.float32, device=self.e.device) if self.e.last else None
        self.xbusy = [False] * self.K
        self.gbusy = [False] * self.K

    def _slot(self, i):
        return self.slots[i % self.K]

    def x_buffer(self, i):
        k = i % self.K
        if self.xbusy[k]:
            raise RuntimeError(f"pipeline activation slot {k} reused before its backward was queued")
        self.xbusy[k] = True
        return self._slot(i)["x"].detach(), k

    def x_input(self, i, slot):
        return self._slot(i)["x"]

    def g_buffer(self, b):
        k = b % self.K
        if self.gbusy[k]:
            raise RuntimeError(f"pipeline gradient slot {k} reused before its backward was queued")
        self.gbusy[k] = True
        return self._slot(b)["g"], k

    def g_input(self, b, slot):
        return self._slot(b)["g"]

    def forward(self, i, x):
        sl = self._slot(i)
        if sl["send_y"] is not None:
            sl["send_y"].wait()  # y_k of micro-batch i - K has left before the replay rewrites it
            sl["send_y"] = None
        for key, v in self.mbs[i].items():
            sl["inp"][key].copy_(v, non_blocking=True)
        sl["step"].copy_(self.steps[i:i + 1])
        sl["gf"].replay()
        self.e.stats["replays"] += 1
        self.e.stats["fwd"] += 1
        if self.e.last:
            self.loss.add_(sl["y"].detach())
        return sl["y"]

    def backward(self, b, y, x, g):
        sl = self._slot(b)
        if sl["send_gx"] is not None:
            sl["send_gx"].wait()
            sl["send_gx"] = None
        sl["gb"].replay()
        self.e.stats["replays"] += 1
        self.e.stats["bwd"] += 1
        return sl["gx"]

    def send_y(self, i, pend):
        self._slot(i)["send_y"] = pend
        return None  # waited per slot (and at the end of the step via finish)

    def send_gx(self, b, pend):
        self._slot(b)["send_gx"] = pend
        return None

    def release_x(self, b, x, slot):
        if slot is not None:
            self.xbusy[slot] = False

    def release_g(self, slot):
        self.gbusy[slot] = False

    def finish(self):
        for sl in self.slots:  # every send of this step has completed before the optimizer step
            for key in ("send_y", "send_gx"):
                if sl[key] is not None:
                    sl[key].wait()
                    sl[key] = None
        return self.loss


class _ChunkGraphRun:
    """Replay-based compute of one interleaved ``train_batch``: micro-batch i of chunk c replays
    slot (c, i mod K_c); a slot's static output (y, or dX) is rewritten only after the send that
    read it completed, a slot is handed to a new micro-batch only after the old one's backward was
    queued (raises otherwise)."""

    def __init__(self, gr, slots, mbs, gscale, micro_step0):
        self.gr, self.e, self.mbs = gr, gr.e, mbs
        self.slots = slots
        self.nvs = self.e.S * self.e.V
        gr.gs.copy_(gscale.reshape(()))
        self.steps = torch.arange(micro_step0, micro_step0 + len(mbs), dtype=torch.int64).to(
            self.e.device, non_blocking=True)
        self.loss = torch.zeros((), dtype=torch.float32, device=self.e.device) if self.e.last else None
        self.owner = [[None] * len(sl) for sl in slots]  # micro-batch holding each slot

    def _k(self, c, i):
        return i % len(self.slots[c])

    def _claim(self, c, i):
        k = self._k(c, i)
        o = self.owner[c][k]
        if o is not None and o != i:
            raise RuntimeError(f"pipeline chunk {c} slot {k} reused by micro-batch {i} before the backward "
                               f"of micro-batch {o} was queued")
        self.owner[c][k] = i
        return self.slots[c][k]

    def x_buffer(self, c, i):
        return self._claim(c, i)["x"].detach(), self._k(c, i)

    def g_buffer(self, c, i):
        return self._claim(c, i)["g"], self._k(c, i)

    def forward(self, c, i, xslot):
        sl = self._claim(c, i)
        if sl["send_y"] is not None:
            sl["send_y"].wait()  # the previous occupant's output has left before the replay rewrites it
            sl["send_y"] = None
        for key, v in self.mbs[i].items():
            sl["inp"][key].copy_(v, non_blocking=True)
        sl["step"].copy_(self.steps[i:i + 1])
        sl["gf"].replay()
        self.e.stats["replays"] += 1
        self.e.stats["fwd"] += 1
        if c * self.e.S + self.e.s == self.nvs - 1:
            self.loss.add_(sl["y"].detach())
        return sl["y"]

    def backward(self, c, i, g):
        sl = self._claim(c, i)
        if sl["send_gx"] is not None:
            sl["send_gx"].wait()
            sl["send_gx"] = None
        sl["gb"].replay()
        self.e.stats["replays"] += 1
        self.e.stats["bwd"] += 1
        return sl["gx"]

    def send_y(self, c, i, pend):
        self.slots[c][self._k(c, i)]["send_y"] = pend
        return None

    def send_gx(self, c, i, pend):
        self.slots[c][self._k(c, i)]["send_gx"] = pend
        return None

    def release_x(self, c, i):
        self.owner[c][self._k(c, i)] = None

    def release_g(self, c, i, slot):
        pass  # the gradient buffer lives in the slot, freed with it by release_x

    def finish(self):
        for chunk in self.slots:
            for sl in chunk:
                for key in ("send_y", "send_gx"):
                    if sl[key] is not None:
                        sl[key].wait()
                        sl[key] = None
        return self.loss


def schedule_1f1b(S, s, M):
    """Pure description of stage s's op order: [('F', i) | ('B', i)] (for tests / docs)."""
    nwarm = min(S - s - 1, M)
    ops = [("F", i) for i in range(nwarm)]
    b = 0
    for j in range(M - nwarm):
        ops.append(("F", nwarm + j))
        ops.append(("B", b))
        b += 1
    ops += [("B", b + k) for k in range(nwarm)]
    return ops


def gather_adapter_state(model, ctx):
    """Full PEFT adapter state on global rank 0 (every stage of replica 0 contributes its
    own LoRA tensors); {} elsewhere.  Collective over the gloo control group."""
    import torch.distributed as dist
    from ..lora import adapter_state_dict
    mine = adapter_state_dict(model) if ctx.dp_rank == 0 else {}
    if ctx.world == 1 or not dist.is_initialized():
        return mine
    parts = [None] * ctx.world
    dist.all_gather_object(parts, mine, group=ctx.ctrl_group)
    if ctx.rank != 0:
        return {}
    full = {}
    for p in parts:
        full.update(p)
    return full
