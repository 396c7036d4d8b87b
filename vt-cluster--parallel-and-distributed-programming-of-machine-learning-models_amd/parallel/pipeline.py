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
  * adjacent-stage transfers are one grouped ``batch_isend_irecv`` per
    exchange (send-activation + recv-gradient together), which RCCL runs on
    its own stream over the direct xGMI link between the two GPUs.

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
        self.p2p = P2P()
        self.dtype, self.d = act_dtype, hidden_size
        self.device = ctx.device
        self.stats = {"fwd": 0, "bwd": 0}

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

    # ---- p2p ----
    def _recv_fwd(self, mb):
        if self.first:
            return None
        x = torch.empty(self._act_shape(mb), dtype=self.dtype, device=self.device)
        self.p2p.exchange(recvs=[(x, self.prev)])
        return x.requires_grad_(True)

    def _send_fwd(self, y):
        if not self.last:
            self.p2p.exchange(sends=[(y.detach().contiguous(), self.next)])

    def _send_fwd_recv_bwd(self, y, mb):
        if self.last:
            return None
        g = torch.empty(self._act_shape(mb), dtype=self.dtype, device=self.device)
        self.p2p.exchange(sends=[(y.detach().contiguous(), self.next)], recvs=[(g, self.next)])
        return g

    def _recv_bwd(self, mb):
        if self.last:
            return None
        g = torch.empty(self._act_shape(mb), dtype=self.dtype, device=self.device)
        self.p2p.exchange(recvs=[(g, self.next)])
        return g

    def _send_bwd(self, gx):
        if not self.first:
            self.p2p.exchange(sends=[(gx.contiguous(), self.prev)])

    def _send_bwd_recv_fwd(self, gx, mb_next):
        if self.first:
            return None
        x = torch.empty(self._act_shape(mb_next), dtype=self.dtype, device=self.device)
        self.p2p.exchange(sends=[(gx.contiguous(), self.prev)], recvs=[(x, self.prev)])
        return x.requires_grad_(True)

    # ---- schedule ----
    def train_batch(self, mbs, gscale, micro_step0):
        """1F1B over ``mbs`` (already on device).  Returns the summed loss (last stage) or None.

        micro-batch i runs with ``model.micro_step = micro_step0 + i`` on every
        stage, so dropout masks are identical to the non-pipelined run."""
        M = len(mbs)
        nwarm = min(self.S - self.s - 1, M)
        nsteady = M - nwarm
        live = deque()
        loss_acc = torch.zeros((), dtype=torch.float32, device=self.device) if self.last else None

        def fwd(i, x):
            y = self._forward(mbs[i], x, micro_step0 + i)
            if self.last:
                loss_acc.add_(y.detach())
            return y

        for i in range(nwarm):
            x = self._recv_fwd(mbs[i])
            y = fwd(i, x)
            self._send_fwd(y)
            live.append((x, y))
        x = self._recv_fwd(mbs[nwarm]) if nsteady > 0 else None
        for j in range(nsteady):
            i = nwarm + j
            y = fwd(i, x)
            g = self._send_fwd_recv_bwd(y, mbs[i - nwarm])  # grad of the oldest live micro-batch
            live.append((x, y))
            bx, by = live.popleft()
            gx = self._backward(by, bx, g, gscale)
            if j == nsteady - 1:
                self._send_bwd(gx)
                x = None
            else:
                x = self._send_bwd_recv_fwd(gx, mbs[i + 1])
        for k in range(nwarm):
            bi = nsteady + k
            g = self._recv_bwd(mbs[bi])
            bx, by = live.popleft()
            gx = self._backward(by, bx, g, gscale)
            self._send_bwd(gx)
        return loss_acc


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
