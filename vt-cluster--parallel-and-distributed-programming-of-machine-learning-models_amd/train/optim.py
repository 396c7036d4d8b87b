"""Fused AdamW + global-norm clip + dynamic loss scaling over a flat arena.

One object drives both execution paths with identical semantics:
  * GPU: two HIP launches (csrc/kernels/adamw.hip ``opt_stats`` + ``opt_apply``), no host sync and
    no per-step device fill: the learning rate is a launch argument, the clip / found-inf / loss-scale
    finalize runs inside one of the two launches (after the stats all-reduce when there is one);
  * CPU: the same math in torch ops (reference / world_size=1 plumbing).

State tensor layout (device, fp32): [step, loss_scale, good_steps,
clip_coef, found_inf, grad_norm].  Reading it (``.stats()``) is the only
host sync and is done only at logging steps.

``reduce_stats_group``: for pipeline parallel the LoRA tensors are split
over stages and for ZeRO-1 over DP ranks, so sum(g^2) and the non-finite
flag are all-reduced over that group before the finalize step (reference
X12: DeepSpeed's model-parallel grad-norm all-reduce).
"""
import math

import torch
import torch.distributed as dist

from ..ops.dispatch import use_kernels, C


class FusedAdamW:
    def __init__(self, params: torch.Tensor, grads: torch.Tensor, lr: float = 5e-5, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, max_grad_norm: float = 1.0,
                 loss_scale: str = "none", init_scale: float = 2.0 ** 16, growth_interval: int = 2000,
                 reduce_stats_group=None, n_valid=None):
        assert params.dtype == torch.float32 and grads.dtype == torch.float32
        self.p, self.g = params, grads
        self.m = torch.zeros_like(params)
        self.v = torch.zeros_like(params)
        self.betas, self.eps, self.wd = betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.dynamic = loss_scale == "dynamic"
        dev = params.device
        self.lr = float(lr)
        self.base_lr = lr
        scale = init_scale if self.dynamic else 1.0
        self.state = torch.tensor([0.0, scale, 0.0, 1.0, 0.0, 0.0], dtype=torch.float32, device=dev)
        self.stats_buf = torch.zeros(2, dtype=torch.float32, device=dev)
        from ..ops.kernels import ARRIVE_INTS
        # the kernels' self-resetting arrival counters: opt_stats' set, then opt_apply's counter
        self.ws = torch.zeros(ARRIVE_INTS + 32, dtype=torch.int32, device=dev)
        self.growth_interval = growth_interval
        # sum(g^2) / non-finite count are summed over every group holding a disjoint part
        # of the parameters (pipeline stages, ZeRO-1 shards)
        g = reduce_stats_group
        self.groups = [x for x in (g if isinstance(g, (list, tuple)) else [g]) if x is not None]
        self.kernels = use_kernels(params)

    # ---- scaling ----
    @property
    def loss_scale_t(self):
        return self.state[1:2]

    def set_lr(self, lr: float):
        self.lr = float(lr)

    def step(self):
        reduce = dist.is_initialized() and bool(self.groups)
        if self.kernels:
            K = C()
            fin = (float(self.max_grad_norm or 0.0), self.dynamic, 2.0, 0.5, self.growth_interval)
            # no all-reduce of the stats: finalize inside opt_stats; else inside opt_apply
            K.opt_stats(self.g, self.stats_buf, self.ws, self.state, not reduce, *fin)
            if reduce:
                for grp in self.groups:
                    dist.all_reduce(self.stats_buf, group=grp)
            K.opt_apply(self.p, self.g, self.m, self.v, self.lr, self.state, self.stats_buf, self.ws, reduce, *fin,
                        self.betas[0], self.betas[1], self.eps, self.wd)
            return
        self.stats_buf[0] = (self.g * self.g).sum()
        self.stats_buf[1] = (~torch.isfinite(self.g)).sum().float()
        if reduce:
            for grp in self.groups:
                dist.all_reduce(self.stats_buf, group=grp)
        self._finalize_ref()
        self._adamw_ref()

    def _finalize_ref(self):
        s = self.state
        scale = s[1].item()
        inf = (self.stats_buf[1].item() != 0.0) or not math.isfinite(self.stats_buf[0].item())
        norm = math.sqrt(max(self.stats_buf[0].item(), 0.0)) / scale
        coef = 1.0 / scale
        if self.max_grad_norm and norm > self.max_grad_norm:
            coef = coef * (self.max_grad_norm / (norm + 1e-6))
        s[3], s[4], s[5] = coef, 1.0 if inf else 0.0, norm
        if not inf:
            s[0] += 1
        if self.dynamic:
            if inf:
                s[1] = max(scale * 0.5, 1.0)
                s[2] = 0
            else:
                s[2] += 1
                if s[2].item() >= self.growth_interval:
                    s[1] = scale * 2.0
                    s[2] = 0

    @torch.no_grad()
    def _adamw_ref(self):
        s = self.state
        if s[4].item() != 0.0:
            self.g.zero_()
            return
        b1, b2 = self.betas
        step = s[0].item()
        lr = torch.tensor(self.lr, dtype=torch.float32).item()  # fp32 lr, as the kernel sees it
        g = self.g * s[3]
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        denom = (self.v.sqrt() / math.sqrt(bc2)).add_(self.eps)
        self.p.mul_(1 - lr * self.wd)
        self.p.addcdiv_(self.m, denom, value=-lr / bc1)
        self.g.zero_()

    def stats(self):
        """Host copy of (step, loss_scale, grad_norm, found_inf) — syncs."""
        s = self.state.tolist()
        return {"step": int(s[0]), "loss_scale": s[1], "grad_norm": s[5], "found_inf": bool(s[4])}

    def state_dict(self):
        return {"m": self.m.cpu(), "v": self.v.cpu(), "state": self.state.cpu(),
                "lr": torch.tensor([self.lr], dtype=torch.float32)}

    def load_state_dict(self, sd):
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.state.copy_(sd["state"])
        self.lr = float(sd["lr"].reshape(-1)[0])


def linear_schedule(base_lr: float, total_steps: int, warmup: int = 0):
    """HF `get_linear_schedule_with_warmup` (reference: no warmup, decay to 0).

    Returns lr for the *next* optimizer step index (0-based), matching the
    Trainer, which logs lr 0.000496 at step 1 of 125 from 5e-4
    (slurm_logs/train.8049.out:8)."""
    def f(step):
        if warmup and step < warmup:
            return base_lr * float(step) / float(max(1, warmup))
        return base_lr * max(0.0, float(total_steps - step) / float(max(1, total_steps - warmup)))
    return f
