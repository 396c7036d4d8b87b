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
  * adjacent-stage transfers are ``batch_isend_irecv`` posts on one
    communicator per direction (activations forward, gradients backward), so
    a receive can be posted ahead of the compute that needs it without ever
    queueing behind the other direction's send; RCCL runs them on their own
    streams over the direct xGMI link, into reused ring buffers.

Loss normalisation: the last stage scales each micro-batch's summed token
loss by ``loss_scale / global_ntokens`` (token-count normalisation over the
whole optimizer step and all DP replicas), so PP, DP and single-GPU runs
produce the same update for the same data.
"""
from collections import deque

import torch

from .comm import P2P


def partition_layers(n_layers, n_stages, method="uniform", head_layers=0.0, embed_layers=0.0):
    """-> list of per-stage layer counts (sum = n_layers)."""
    if n_stages > n_layers:
        raise ValueError(f"{n_stages} stages > {n_layers} layers")
    if method == "uniform":
        return [n_layers // n_stages + (1 if i < n_layers % n_stages else 0) for i in range(n_stages)]
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


def stage_layer_range(split, stage):
    lo = sum(split[:stage])
    return lo, lo + split[stage]


def head_cost_layers(cfg):
    """LM-head MACs in units of one decoder layer (12·d² MACs per token + attention ignored)."""
    d = getattr(cfg, "hidden_size", None) or getattr(cfg, "n_embd")
    ffn = getattr(cfg, "ffn_dim", None) or getattr(cfg, "n_inner", 4 * d)
    return cfg.vocab_size * d / (4 * d * d + 2 * d * ffn)


class PipelineEngine:
    """Runs one optimizer step's micro-batches through this rank's stage.

    ``model``: the stage model (``has_embed`` on stage 0, ``has_head`` on the
    last).  ``ctx``: mift.parallel.dist.DistContext (pp_rank, pp_ranks, ...)."""

    def __init__(self, model, ctx, act_dtype, hidden_size):
        self.model, self.ctx = model, ctx
        self.S, self.s = ctx.pp, ctx.pp_rank
        self.first, self.last = self.s == 0, self.s == self.S - 1
        self.prev = ctx.pp_ranks[self.s - 1] if not self.first else None
        self.next = ctx.pp_ranks[self.s + 1] if not self.last else None
        # one communicator per direction: activations (s -> s+1) and their grads (s+1 -> s)
        self.p2p_f = P2P(getattr(ctx, "pp_fwd_group", None))
        self.p2p_b = P2P(getattr(ctx, "pp_bwd_group", None))
        self.dtype, self.d = act_dtype, hidden_size
        self.device = ctx.device
        self.stats = {"fwd": 0, "bwd": 0}
        # receive rings: an activation lives until its micro-batch's backward (at most S - s in
        # flight on stage s) plus the one prefetched ahead; a gradient only until its backward
        self._xring = _Ring(self.S - self.s + 1, act_dtype, self.device)
        self._gring = _Ring(2, act_dtype, self.device)

    # ---- per-micro-batch compute ----
    def _act_shape(self, mb):
        b, S = mb["input_ids"].shape
        return (b, S, self.d)

    def _forward(self, mb, x, micro_step):
        m = self.model
        m.micro_step = micro_step
        out = m(input_ids=mb["input_ids"] if self.first else None, attention_mask=mb["attention_mask"],
                labels=mb["labels"] if self.last else None, hidden_states=x, reduction="sum",
                return_logits=False)
        self.stats["fwd"] += 1
        return out["loss"].float() if self.last else out["hidden_states"]

    def _backward(self, y, x, grad_y, gscale):
        if self.last:
            (y * gscale).backward()
        else:
            torch.autograd.backward(y, grad_tensors=grad_y)
        self.stats["bwd"] += 1
        return x.grad if x is not None else None

    # ---- schedule ----
    def train_batch(self, mbs, gscale, micro_step0):
        """1F1B over ``mbs`` (already on device).  Returns the summed loss (last stage) or None.

        micro-batch i runs with ``model.micro_step = micro_step0 + i`` on every
        stage, so dropout masks are identical to the non-pipelined run.

        Communication is asynchronous and posted AHEAD of the compute that needs it:
        the activation of micro-batch i+1 is requested before micro-batch i's forward runs,
        and the gradient for the next backward before the forward that precedes it, each
        into a reusable ring buffer.  Sends are fire-and-forget until the end of the step.
        On RCCL ``Pending.wait()`` only orders the compute stream behind the transfer, so
        the host never blocks and xGMI transfers overlap the forward / backward kernels."""
        M = len(mbs)
        nwarm = min(self.S - self.s - 1, M)
        nsteady = M - nwarm
        live = deque()
        xq = deque()
        sends = []
        loss_acc = torch.zeros((), dtype=torch.float32, device=self.device) if self.last else None

        def post_x(i):
            if not self.first and i < M:
                buf = self._xring.get(self._act_shape(mbs[i]))
                xq.append(self.p2p_f.post(recvs=[(buf, self.prev)]))

        def take_x():
            if self.first:
                return None
            return xq.popleft().wait()[0].requires_grad_(True)

        def post_g(b):
            if self.last:
                return None
            return self.p2p_b.post(recvs=[(self._gring.get(self._act_shape(mbs[b])), self.next)])

        def fwd(i, x):
            y = self._forward(mbs[i], x, micro_step0 + i)
            if self.last:
                loss_acc.add_(y.detach())
            else:
                sends.append(self.p2p_f.post(sends=[(y.detach(), self.next)]))
            return y

        def bwd(gp):
            bx, by = live.popleft()
            g = gp.wait()[0] if gp is not None else None
            gx = self._backward(by, bx, g, gscale)
            if not self.first:
                sends.append(self.p2p_b.post(sends=[(gx, self.prev)]))
                bx.grad = None  # the ring slot is reused by a later micro-batch

        post_x(0)
        for i in range(nwarm):
            x = take_x()
            post_x(i + 1)
            live.append((x, fwd(i, x)))
        for j in range(nsteady):
            i = nwarm + j
            gp = post_g(j)          # grad of the oldest live micro-batch, requested before the forward
            x = take_x()
            post_x(i + 1)
            live.append((x, fwd(i, x)))
            bwd(gp)
        for k in range(nwarm):
            bwd(post_g(nsteady + k))
        for p in sends:
            p.wait()
        return loss_acc


class _Ring:
    """Receive buffers reused round-robin per shape (``n`` slots: the in-flight bound)."""

    def __init__(self, n, dtype, device):
        self.n, self.dtype, self.device = max(1, n), dtype, device
        self.bufs, self.idx = {}, {}

    def get(self, shape):
        shape = tuple(shape)
        bufs = self.bufs.setdefault(shape, [])
        i = self.idx.get(shape, 0)
        self.idx[shape] = i + 1
        if len(bufs) < self.n:
            bufs.append(torch.empty(shape, dtype=self.dtype, device=self.device))
        # a fresh leaf view per use: no autograd state (.grad, requires_grad) carries over
        return bufs[i % self.n].detach()


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
