"""Data-parallel LoRA trainer (replaces HF Trainer + torch DDP, reference C16/C21/C35).

Semantics kept from the reference (HF Trainer defaults):
  * per-rank micro-batch ``batch`` x ``accum`` micro-steps per optimizer step;
  * loss normalised by the number of label tokens in the whole optimizer
    step across all DP ranks (Trainer's ``num_items_in_batch`` path), so
    ``batch=1, accum=32`` and ``batch=32, accum=1`` give the same update;
  * AdamW(β=(0.9,0.999), eps 1e-8, wd 0), global-norm clip 1.0, linear LR
    decay to 0 with no warmup;
  * ``no_sync`` on accumulation micro-steps, one gradient all-reduce per
    optimizer step;
  * step / phase log lines in the reference formats (mift.obs.timing);
  * checkpoint-N dirs every ``save_steps`` (adapter, optimizer, rng,
    trainer_state.json, data position) + ``resume='auto'``.

MI355X-specific: bf16 (default) / fp16 with device-side dynamic loss scaling
/ fp32; the optimizer step, clip and loss scale never sync the host; the
host only syncs at logging steps.
"""
import json
import math
import os
import shutil
import time
from dataclasses import dataclass, asdict, field
from typing import Optional

import torch
import torch.distributed as dist

from ..lora import LoraArena, adapter_state_dict, save_adapter
from ..obs.profiler import StepProfiler, parse_window, rng
from ..obs.timing import HOST, hf_log_line, lab_step_line, p1_step_line, perf_line
from ..parallel.ddp import GradReducer, verify_replicas
from ..utils.faults import maybe_inject
from .optim import FusedAdamW, linear_schedule


@dataclass
class TrainConfig:
    epochs: float = 1.0
    batch: int = 1
    accum: int = 32
    lr: float = 5e-5
    warmup_steps: int = 0
    weight_decay: float = 0.0
    max_grad_norm: float = 1.0
    precision: str = "bf16"           # bf16 | fp16 | fp32
    logging_steps: int = 50
    save_steps: int = 500
    save_total_limit: int = 1
    max_steps: int = -1
    seed: int = 0
    output_dir: Optional[str] = None
    resume: Optional[str] = None       # None | 'auto' | path
    step_log: str = "p1"               # p1 | lab | none
    bucket_mb: float = 25.0
    recompute: bool = False
    shuffle: bool = False
    zero_stage: int = 0                # 1: shard AdamW state over the DP group (mift.parallel.zero)
    trainable: str = "lora"            # lora | all (full fine-tuning: the tiny-BERT lab)
    logging_first_step: bool = False
    graph: str = "auto"                # hipGraph-replayed steps (mift.train.graph): auto | on | off (MIFT_GRAPH)
    consistency_every: int = 0         # >0: checksum the trainable params across DP replicas every N steps
    consistency_rtol: float = 1e-5     # periodic check: ulp-level drift tolerated (and healed), see verify_replicas
    max_inflight_steps: int = 2        # host run-ahead bound (GPU): wait for step i-N before returning from step i
    profile_dir: Optional[str] = None  # torch.profiler window (mift.obs.profiler): trace/kernels/ranges per rank
    profile_steps: str = "3:6"         # global steps [A, B) recorded when profile_dir is set
    warm_setup: bool = True            # GPU graph path: eager warm-up + capture at construction (MIFT_WARM_SETUP)


class Trainer:
    def __init__(self, model, batcher, cfg: TrainConfig, ctx=None, callbacks=(), epoch_callbacks=()):
        self.model, self.batcher, self.cfg, self.ctx = model, batcher, cfg, ctx
        self.rank = ctx.rank if ctx else 0
        self.device = ctx.device if ctx else torch.device("cpu")
        self.dp_group = ctx.dp_group if ctx else None
        self.dp = ctx.dp if ctx else 1
        self.pp = ctx.pp if ctx else 1
        self.zero = cfg.zero_stage >= 1 and self.dp > 1
        named = None
        if cfg.trainable == "all":
            named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        self.arena = LoraArena(model, device=self.device, shards=self.dp if self.zero else 1, named=named)
        if self.device.type == "cuda" and getattr(model, "fused", False) and named is None:
            from ..lora.pack import attach
            from ..ops.dispatch import use_kernels
            if use_kernels(self.arena.param):
                attach(model, self.arena, next(p for n, p in model.named_parameters() if "lora_" not in n).dtype)
        okw = dict(lr=cfg.lr, weight_decay=cfg.weight_decay, max_grad_norm=cfg.max_grad_norm,
                   loss_scale="dynamic" if cfg.precision == "fp16" else "none")
        pp_group = ctx.pp_group if (ctx and self.pp > 1) else None
        if self.zero:
            from ..parallel.zero import Zero1AdamW
            self.reducer = None
            self.opt = Zero1AdamW(self.arena, self.dp_group, self.dp, ctx.dp_rank, stats_groups=[pp_group], **okw)
        else:
            # PP interleaves micro-batch backwards, so its DP all-reduce runs once after the schedule
            self.reducer = GradReducer(self.arena, group=self.dp_group, bucket_mb=cfg.bucket_mb, world=self.dp,
                                       overlap=self.pp == 1)
            self.opt = FusedAdamW(self.arena.param, self.arena.grad, reduce_stats_group=pp_group, **okw)
        self.engine = None
        if self.pp > 1:
            from ..parallel.pipeline import PipelineEngine
            act_dtype = next(p for n, p in model.named_parameters() if "lora_" not in n).dtype
            if self.device.type == "cpu" and cfg.precision == "bf16":
                act_dtype = torch.float32
            hidden = getattr(model.config, "hidden_size", None) or model.config.n_embd
            self.engine = PipelineEngine(model, ctx, act_dtype, hidden, graph=self._fused_graphable("pipeline"))
        spe = batcher.steps_per_epoch()
        self.steps_per_epoch = spe
        total = int(math.ceil(spe * cfg.epochs))
        if cfg.max_steps > 0:
            total = min(total, cfg.max_steps)
        self.total_steps = total
        self.sched = linear_schedule(cfg.lr, total, cfg.warmup_steps)
        self.global_step = 0
        self.callbacks = list(callbacks)              # (trainer, log record) at logging steps
        self.epoch_callbacks = list(epoch_callbacks)  # (trainer, epoch) at each epoch end (eval)
        self.history = []
        if hasattr(model, "recompute"):
            model.recompute = cfg.recompute
        self._ctrl = ctx.ctrl_group if ctx else None
        self.graphed = None
        if self._graph_ok():
            from .graph import GraphedStep
            self.graphed = GraphedStep(self)
        self._comm_ev = None
        self._inflight = []  # completion events of the optimizer steps still queued on the GPU
        self._tok_seen = 0
        if self.dp > 1 and dist.is_initialized():
            # replaces DDP's construction broadcast (reference X6): identical init by seed,
            # verified with one checksum all-reduce over the DP group
            verify_replicas([self.arena.param] + [p.detach() for p in model.parameters() if not p.requires_grad],
                            group=self.dp_group)
        if self.graphed is not None and os.environ.get("MIFT_WARM_SETUP", "1" if cfg.warm_setup else "0") != "0":
            self._warm_setup()

    def _warm_setup(self):
        """Pay the one-time costs at construction (the reference's ``[Trainer setup]`` phase) instead
        of inside the first training steps: one eager forward+backward on a full-shape sample step
        (first launch of every kernel module, allocator growth, LoRA pack), then the hipGraph
        capture of that shape, so step 1 already replays.  Nothing of it reaches training state:
        the micro-step counter (dropout seeds) is restored, the grads are zeroed, no collective runs
        (DP bucket all-reduces are suppressed) and the optimizer is not stepped.  Measured by
        tools/coldstart.py (~1.3 s of first-steps cost inside [Training])."""
        model, g = self.model, self.graphed
        mbs = self.batcher.sample_step()
        sig = g.signature(mbs)
        ms0 = model.micro_step
        was_training = model.training
        model.train()
        red = self.reducer
        gscale = (self.opt.loss_scale_t / 1.0e6).reshape(())
        with (red.no_sync() if red is not None else _null()):
            for mb in mbs:
                mb = self._to_dev(mb)
                model.next_micro_step()
                out = model(input_ids=mb["input_ids"], attention_mask=mb["attention_mask"], labels=mb["labels"],
                            reduction="sum", return_logits=False)
                out["loss"].float().backward(gscale)
        from ..ops.fused import reset_wgrads
        reset_wgrads()
        from ..ops.dispatch import C
        C().grad_stats(self.opt.g, self.opt.stats_buf)  # first launch of the optimizer kernels' module
        model.micro_step = ms0
        g.seen.add(sig)
        g.prepare(mbs)
        if os.environ.get("MIFT_DIAG_NOREBIND") != "1":
            self.arena.rebind_grads()
        self.arena.grad.zero_()
        if red is not None:
            red.begin_step()
        model.train(was_training)
        torch.cuda.synchronize(self.device)

    def _fused_graphable(self, what):
        """hipGraph replay applies: the fused GPU LoRA path without recompute (``graph`` auto|on|off,
        env MIFT_GRAPH).  ``what``: "step" (whole-step graph, pp = 1) or "pipeline" (per-slot stage
        graphs of the PP engine)."""
        mode = os.environ.get("MIFT_GRAPH", self.cfg.graph)
        if mode in ("off", "0", "false", False, "", None) or self.device.type != "cuda":
            return False
        from ..ops.dispatch import use_kernels
        ok = (getattr(self.model, "fused", False) and use_kernels(self.arena.param)
              and self.cfg.trainable == "lora" and not self.cfg.recompute and hasattr(self.model, "micro_step"))
        if mode in ("on", "1", "true", True) and not ok:
            raise RuntimeError("graph=on needs the fused GPU LoRA path without recompute")
        return ok

    def _replicated_opt_state(self):
        """The optimizer tensors laid out like the full arena and identical on every DP replica (the
        AdamW moments), resynchronised together with the parameters; ZeRO-1 shards them per rank."""
        if self.cfg.zero_stage:
            return []
        return [t for t in (getattr(self.opt, "m", None), getattr(self.opt, "v", None))
                if t is not None and t.numel() == self.arena.param.numel()]

    def _graph_ok(self):
        return self.pp == 1 and self._fused_graphable("step")

    # ------------------------------------------------------------------
    def _global_tokens(self, mbs):
        count = getattr(self.model, "count_targets", None)
        pre = getattr(mbs, "global_tokens", None)
        if count is None and pre is not None:
            # causal LM: precomputed from the deterministic shard plan (MicroBatcher.global_step_tokens),
            # so the step issues no blocking control-plane all-reduce
            return max(int(pre), 1)
        if count is not None:  # e.g. sequence classification: one target per row
            n = sum(count(mb["labels"]) for mb in mbs)
        else:  # causal LM: shifted label tokens
            n = sum(int((mb["labels"][:, 1:] != -100).sum()) for mb in mbs)
        if self.dp > 1 and dist.is_initialized():
            t = torch.tensor([n], dtype=torch.float64)
            dist.all_reduce(t, group=self._dp_ctrl_group())
            n = int(t.item())
        return max(n, 1)

    def _dp_ctrl_group(self):
        if not hasattr(self, "_dpc"):
            self._dpc = None
            if self.ctx is not None and self.ctx.dp > 1:
                if self.ctx.pp == 1:
                    self._dpc = self.ctx.ctrl_group
                else:
                    # gloo mirror of the DP group (created collectively on all ranks)
                    groups = {}
                    for s in range(self.ctx.pp):
                        ranks = list(range(s, self.ctx.world, self.ctx.pp))
                        groups[s] = dist.new_group(ranks, backend="gloo", timeout=self.ctx.timeout)
                    self._dpc = groups[self.ctx.pp_rank]
        return self._dpc

    def _to_dev(self, mb):
        return {k: v.to(self.device, non_blocking=True) for k, v in mb.items()}

    def train_step(self, mbs):
        """One optimizer step over a list of micro-batches. Returns loss_sum tensor.

        The host may run at most ``max_inflight_steps`` optimizer steps ahead of the GPU: measured on
        MI355X, an unbounded queue of graph replays + input copies + optimizer launches slowed the
        distilgpt2 step from 4.96 to 5.40 ms (bench.py, same box), while a bound of 1-4 steps keeps
        the GPU fed (the host needs ~0.3 ms per step to enqueue one) at 4.95-4.96 ms."""
        with rng("mift.step"):
            out = self._train_step(mbs)
        self._bound_inflight()
        return out

    def _bound_inflight(self):
        n = int(self.cfg.max_inflight_steps)
        if n <= 0 or self.device.type != "cuda":
            return
        ev = torch.cuda.Event()
        ev.record()
        self._inflight.append(ev)
        while len(self._inflight) > n:
            self._inflight.pop(0).synchronize()

    def _train_step(self, mbs):
        model, cfg = self.model, self.cfg
        from ..ops.fused import reset_wgrads
        reset_wgrads()  # a previous step's backward that raised must not leak queued weight grads
        ntok = self._global_tokens(mbs)
        if self.reducer is not None:
            self.reducer.begin_step(self.global_step + 1)
        lr = self.sched(self.global_step)
        self.opt.set_lr(lr)
        if self.graphed is not None and self.graphed.supported(mbs):
            with rng("mift.fwd_bwd.graph"):
                loss = self.graphed.run(mbs, ntok)
            return self._finish_step(loss, ntok)
        # loss_scale * fl32(1/ntok): the exact product the graph replay computes on the device
        # (train/graph.py inv_ntok), so eager and replayed steps see bit-identical upstream grads
        gscale = self.opt.loss_scale_t * (1.0 / ntok)
        if self.engine is not None:
            dev_mbs = [self._to_dev(mb) for mb in mbs]
            ms0 = model.micro_step
            with rng("mift.fwd_bwd.pipeline"):
                loss_acc = self.engine.train_batch(dev_mbs, gscale, ms0 + 1)
            model.micro_step = ms0 + len(mbs)
            maybe_inject(self.rank, self.global_step + 1, "micro")
            return self._finish_step(loss_acc, ntok)
        loss_acc = torch.zeros((), dtype=torch.float32, device=self.device)
        autocast = (self.device.type == "cpu" and cfg.precision == "bf16")
        for i, mb in enumerate(mbs):
            mb = self._to_dev(mb)
            model.next_micro_step()
            last = i == len(mbs) - 1
            ctxm = self.reducer.no_sync() if (not last and self.reducer is not None) else _null()
            with ctxm, rng("mift.fwd_bwd"):
                with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
                    out = model(input_ids=mb["input_ids"], attention_mask=mb["attention_mask"],
                                labels=mb["labels"], reduction="sum", return_logits=False)
                loss_sum = out["loss"].float()
                loss_sum.backward(gscale.reshape(()))
            loss_acc += loss_sum.detach()
            maybe_inject(self.rank, self.global_step + 1, "micro")
        res = self._finish_step(loss_acc, ntok)
        if self.graphed is not None:
            self.graphed.prepare(mbs)  # capture now: the next step of this shape replays
        return res

    def _finish_step(self, loss_acc, ntok):
        self.arena.rebind_grads()
        timed = self.device.type == "cuda" and self.dp > 1
        if timed:
            if self._comm_ev is None:
                self._comm_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self._comm_ev[0].record()
        maybe_inject(self.rank, self.global_step + 1, "grads", grads=self.arena.grad)
        with rng("mift.comm.grads"):
            if self.zero:
                self.opt.reduce_grads()
            else:
                self.reducer.finish()
        if timed:
            self._comm_ev[1].record()
        with rng("mift.optimizer"):
            self.opt.step()
        self.arena.bump()
        self.global_step += 1
        return loss_acc, ntok

    def _loss_for_log(self, loss_sum):
        """Global summed token loss of the step on every rank (sum over DP replicas;
        in PP only the last stage holds a loss, the others contribute 0)."""
        if self.ctx is None or self.ctx.world == 1 or not dist.is_initialized():
            return float(loss_sum)
        t = loss_sum.detach().clone() if loss_sum is not None else torch.zeros((), device=self.device)
        dist.all_reduce(t)
        return float(t)

    # ------------------------------------------------------------------
    def train(self):
        cfg = self.cfg
        start_step = 0
        if cfg.resume:
            start_step = self.resume(cfg.resume)
        self.model.train()
        t_last = time.perf_counter()
        self._perf_t0, self._tok_seen = t_last, 0
        sync_dev = self.device.type == "cuda"
        epoch = start_step // max(1, self.steps_per_epoch)
        done = start_step >= self.total_steps
        prof = (StepProfiler(cfg.profile_dir, self.rank, parse_window(cfg.profile_steps))
                if cfg.profile_dir else None)
        while not done:
            skip = start_step - epoch * self.steps_per_epoch
            for mbs in self.batcher.epoch(epoch, start_step=max(0, skip)):
                if prof is not None:
                    prof.before_step(self.global_step + 1)
                loss_sum, ntok = self.train_step(mbs)
                if prof is not None:
                    prof.after_step(self.global_step)
                maybe_inject(self.rank, self.global_step, "step")
                log_now = bool(cfg.logging_steps) and (self.global_step % cfg.logging_steps == 0 or
                                                       (cfg.logging_first_step and self.global_step == 1))
                if cfg.step_log != "none" or log_now:
                    if sync_dev:
                        torch.cuda.synchronize()
                    now = time.perf_counter()
                    dt = now - t_last
                    t_last = now
                    if cfg.step_log == "p1":
                        print(p1_step_line(self.rank, self.global_step, dt), flush=True)
                    elif cfg.step_log == "lab":
                        samples = cfg.batch * len(mbs) * self.dp
                        sps = samples / max(dt, 1e-9)
                        seq = mbs[0]["input_ids"].shape[1]
                        print(lab_step_line(self.rank, self.global_step, dt * 1000, sps, sps * seq), flush=True)
                self._tok_seen += sum(int(mb["input_ids"].numel()) for mb in mbs) * self.dp
                if cfg.consistency_every and self.dp > 1 and self.global_step % cfg.consistency_every == 0:
                    verify_replicas([self.arena.param], group=self.dp_group, rtol=cfg.consistency_rtol, resync=True,
                                    slices=[[(o, p.numel()) for o, (_, p) in zip(self.arena.offsets, self.arena.named)]],
                                    companions=[self._replicated_opt_state()])
                if log_now:
                    self._perf_log(mbs)
                    st = self.opt.stats()
                    rec = {"loss": self._loss_for_log(loss_sum) / max(1, ntok),
                           "grad_norm": st["grad_norm"], "learning_rate": self.sched(self.global_step),
                           "epoch": round(self.global_step / max(1, self.steps_per_epoch), 4)}
                    self.history.append(dict(rec, step=self.global_step))
                    if self.rank == 0:
                        print(hf_log_line(rec), flush=True)
                    for cb in self.callbacks:
                        cb(self, rec)
                if cfg.output_dir and cfg.save_steps and self.global_step % cfg.save_steps == 0:
                    self.save_checkpoint()
                if self.global_step >= self.total_steps:
                    done = True
                    break
            for cb in self.epoch_callbacks:
                cb(self, epoch)
            epoch += 1
            start_step = epoch * self.steps_per_epoch
            if epoch * self.steps_per_epoch >= self.total_steps:
                done = True
        if prof is not None:
            prof.close()  # window longer than the run: dump what was recorded
        if sync_dev:
            torch.cuda.synchronize()
        return self.history

    def _perf_log(self, mbs):
        if self.rank != 0:
            self._tok_seen, self._perf_t0 = 0, time.perf_counter()
            return
        now = time.perf_counter()
        t0 = getattr(self, "_perf_t0", None)
        self._perf_t0 = now
        toks, self._tok_seen = self._tok_seen, 0
        if t0 is None or now <= t0:
            return
        tps = toks / (now - t0)
        n = getattr(self.model, "num_flop_params", None)
        nparams = n() if callable(n) else sum(p.numel() for p in self.model.parameters())
        tflops = 4.0 * nparams * tps / max(1, self.ctx.world if self.ctx else 1) / 1e12  # fwd + dgrad
        hbm = torch.cuda.max_memory_allocated(self.device) / 2 ** 30 if self.device.type == "cuda" else 0.0
        comm = 0.0
        if self._comm_ev is not None:
            torch.cuda.synchronize(self.device)
            comm = self._comm_ev[0].elapsed_time(self._comm_ev[1])
        print(perf_line(self.rank, self.global_step, tps, tflops, hbm, comm, self.ctx.world if self.ctx else 1),
              flush=True)

    # ------------------------------------------------------------------
    def save_checkpoint(self):
        """``checkpoint-<step>/``: adapter + optimizer + rng + trainer_state (+rotation)."""
        out = os.path.join(self.cfg.output_dir, f"checkpoint-{self.global_step}")
        full = self.cfg.trainable == "all"
        state = {} if full else self.adapter_state()
        if self.rank == 0:
            os.makedirs(out, exist_ok=True)
            if full:
                self.model.save_pretrained(out)
            else:
                save_adapter(out, state, self.model.lora_config)
            with open(os.path.join(out, "trainer_state.json"), "w") as f:
                json.dump({"global_step": self.global_step, "max_steps": self.total_steps,
                           "steps_per_epoch": self.steps_per_epoch, "log_history": self.history,
                           "micro_step": self.model.micro_step, "seed": self.model.seed,
                           "world": self.ctx.world if self.ctx else 1, "dp": self.dp, "pp": self.pp,
                           "zero_stage": int(self.zero)}, f, indent=2)
        if dist.is_initialized():
            dist.barrier(group=self.ctx.ctrl_group if self.ctx else None)
        # Checkpoints live on storage SHARED by every rank (the reference's OUT_ROOT, checked writable
        # from all nodes by its preflight, P1 submit_distilgpt2_lora.sbatch:92-103): rank 0 writes the
        # adapter, trainer_state.json and the DDP optimizer.pt, and every rank reads them on resume.
        # Optimizer state is per rank in PP (stage-local adapters) and ZeRO-1 (shards); plain DDP
        # replicas hold identical state, so only rank 0 writes the shared optimizer.pt.
        os.makedirs(out, exist_ok=True)
        if self._opt_per_rank() or self.rank == 0:
            torch.save(self.opt.state_dict(), os.path.join(out, self._opt_file()))
        torch.save({"cpu": torch.get_rng_state()}, os.path.join(out, f"rng_state_{self.rank}.pth"))
        if dist.is_initialized():
            dist.barrier(group=self.ctx.ctrl_group if self.ctx else None)
        if self.rank == 0 and self.cfg.save_total_limit:
            cks = sorted([d for d in os.listdir(self.cfg.output_dir) if d.startswith("checkpoint-")],
                         key=lambda d: int(d.split("-")[1]))
            for d in cks[:-self.cfg.save_total_limit]:
                shutil.rmtree(os.path.join(self.cfg.output_dir, d), ignore_errors=True)
        return out

    def _opt_per_rank(self):
        return self.pp > 1 or self.zero

    def _opt_file(self):
        return f"optimizer_rank{self.rank}.pt" if self._opt_per_rank() else "optimizer.pt"

    def adapter_state(self):
        """Full PEFT adapter state (gathered over pipeline stages) on rank 0."""
        if self.pp > 1:
            from ..parallel.pipeline import gather_adapter_state
            return gather_adapter_state(self.model, self.ctx)
        return adapter_state_dict(self.model) if self.rank == 0 else {}

    def resume(self, spec):
        path = spec
        if spec == "auto":
            if not self.cfg.output_dir or not os.path.isdir(self.cfg.output_dir):
                return 0
            cks = [d for d in os.listdir(self.cfg.output_dir) if d.startswith("checkpoint-")]
            if not cks:
                return 0
            path = os.path.join(self.cfg.output_dir, max(cks, key=lambda d: int(d.split("-")[1])))
        if self.cfg.trainable == "all":
            from ..models import load_hf_weights
            load_hf_weights(self.model, path)
        else:
            from ..lora import load_adapter
            load_adapter(self.model, path)
        self.opt.load_state_dict(torch.load(os.path.join(path, self._opt_file()), weights_only=True))
        with open(os.path.join(path, "trainer_state.json")) as f:
            st = json.load(f)
        self.global_step = st["global_step"]
        self.history = st.get("log_history", [])
        self.model.micro_step = st.get("micro_step", 0)
        self.arena.bump()
        rp = os.path.join(path, f"rng_state_{self.rank}.pth")
        if os.path.exists(rp):
            torch.set_rng_state(torch.load(rp, weights_only=True)["cpu"])
        if self.rank == 0:
            print(f"[resume] from {path} at step {self.global_step}", flush=True)
        return self.global_step


@torch.no_grad()
def _noop():
    pass


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
