"""ZeRO stage 1: AdamW state sharded over the data-parallel group.

Reference: DeepSpeed ``zero_optimization.stage = 1`` in the P2 config
(`P2/finetune_lora_opt_pp.py:185`, `deepspeed_pp_zero1_cpu_activ.json:4`,
SURVEY C19 / X13).  There it is a no-op (DP = 1 in every run); here it is a
real option for the DP×PP grid.

Over the flat LoRA arena this is three steps per optimizer step:
  1. reduce-scatter the fp32 grad arena over the DP group -> my shard,
  2. fused AdamW (+ clip / inf-check, stats summed over DP shards and PP
     stages) on my shard of params + m + v only,
  3. all-gather the updated parameter shards back into every replica.
The arena is padded to ``dp × 64`` elements so shards are equal and aligned.
For LoRA the saving is small (m+v of 11.8 MB per OPT-2.7B stage) — the
option exists for parity and for full-parameter fine-tuning of larger
adapters; reduce-scatter + all-gather move the same bytes as one all-reduce.
"""
import torch

from ..obs.profiler import rng
from ..train.optim import FusedAdamW
from .comm import all_gather_flat, reduce_scatter_flat


class Zero1AdamW:
    def __init__(self, arena, dp_group, dp, dp_rank, stats_groups=(), **opt_kw):
        n = arena.numel
        if n % dp:
            raise ValueError("arena must be built with shards=dp")
        self.arena, self.group, self.dp = arena, dp_group, dp
        self.shard = n // dp
        self.lo, self.hi = dp_rank * self.shard, (dp_rank + 1) * self.shard
        self.gshard = torch.zeros(self.shard, dtype=torch.float32, device=arena.grad.device)
        groups = [dp_group] + [g for g in stats_groups if g is not None]
        self.opt = FusedAdamW(arena.param[self.lo:self.hi], self.gshard, reduce_stats_group=groups, **opt_kw)

    # FusedAdamW-compatible surface used by the Trainer (tests/test_zero_surface_cpu.py checks that
    # every ``self.opt.<name>`` the Trainer touches exists here)
    @property
    def loss_scale_t(self):
        return self.opt.loss_scale_t

    @property
    def g(self):  # this rank's gradient shard (the Trainer's setup warm-up launches grad_stats on it)
        return self.opt.g

    @property
    def stats_buf(self):
        return self.opt.stats_buf

    @property
    def state(self):
        return self.opt.state

    def set_lr(self, lr):
        self.opt.set_lr(lr)

    def reduce_grads(self):
        with rng("mift.comm.zero_rs"):
            reduce_scatter_flat(self.gshard, self.arena.grad, self.group)
        self.arena.grad.zero_()

    def step(self):
        self.opt.step()
        with rng("mift.comm.zero_ag"):
            all_gather_flat(self.arena.param, self.arena.param[self.lo:self.hi].clone(), self.group)

    def stats(self):
        return self.opt.stats()

    def state_dict(self):
        sd = self.opt.state_dict()
        sd["zero1"] = torch.tensor([self.lo, self.hi, self.dp])
        return sd

    def load_state_dict(self, sd):
        sd = dict(sd)
        sd.pop("zero1", None)
        self.opt.load_state_dict(sd)
