"""One typed run configuration: DeepSpeed-compatible JSON keys + MI355X ``mift.*`` keys.

Reference: P2 loads a DeepSpeed JSON (``--ds_cfg``,
``Cluster/Project 2 - Course Project/finetune_lora_opt_pp.py:179-199``; the shipped
``deepspeed_pp_zero1_cpu_activ.json``) whose knobs were otherwise scattered across CLIs, HF
``TrainingArguments`` and ``LoraConfig`` objects.  Here every knob a run can set lives in
:class:`MiftConfig`, parsed from one JSON file:

* DeepSpeed keys honoured: ``train_micro_batch_size_per_gpu``, ``gradient_accumulation_steps``,
  ``zero_optimization.stage``, ``fp16.enabled`` (+ ``initial_scale_power``,
  ``loss_scale_window``), ``bf16.enabled``, ``optimizer.params`` (lr, betas, eps,
  weight_decay), ``gradient_clipping``, ``activation_checkpointing`` and
  ``pipeline`` (``stages``, ``partition_method``);
* DeepSpeed keys accepted with NO effect are reported, never dropped silently:
  ``zero_optimization.cpu_offload`` and the activation-partitioning / CPU-checkpointing knobs
  (288 GB of HBM per MI355X holds weights, optimizer state and activations);
* ``mift`` section (MI355X-specific, defaults sized for one process per GPU over xGMI):
  ``kernels`` (HIP kernels on/off), ``graph`` (hipGraph replay: auto/on/off), ``lmhead``
  (fused | blas), ``bucket_mb`` (DP all-reduce bucket), ``pp_partition`` (uniform | balanced |
  halves: half-layer units),
  ``pp_schedule`` (1f1b), ``micro_batch`` (GPU micro-batch regrouping: an int, or "auto" = the
  pipeline planner ``mift.parallel.plan.choose_micro_batch``), ``virtual_stages`` (interleaved 1F1B
  chunks per pipeline rank: an int, or "auto" = chosen with the micro-batch), ``side_stream``
  (LoRA weight grads on a second stream), ``comm_timeout_s`` (collective watchdog),
  ``consistency_every`` (replica checksum period), ``max_inflight_steps`` (host run-ahead bound);
* anything else is an error unless ``mift.strict`` is false (then a warning).

``MiftConfig.apply_env()`` exports the process-wide toggles (``MIFT_KERNELS``, ``MIFT_GRAPH``,
``MIFT_LMHEAD``, ``MIFT_SIDE_STREAM``, ``MIFT_COMM_TIMEOUT``) the runtime reads.
"""
import json
import os
import warnings
from dataclasses import asdict, dataclass, field
from typing import List, Optional, Tuple

_DS_KNOWN = {
    "train_micro_batch_size_per_gpu", "gradient_accumulation_steps", "train_batch_size", "zero_optimization",
    "fp16", "bf16", "optimizer", "gradient_clipping", "activation_checkpointing", "pipeline", "steps_per_print",
    "wall_clock_breakdown", "mift", "scheduler",
}
_NO_EFFECT = {
    "zero_optimization.cpu_offload": "optimizer state stays in HBM (288 GB per GPU)",
    "zero_optimization.overlap_comm": "DP buckets always launch during backward",
    "zero_optimization.contiguous_gradients": "gradients always live in one flat arena",
    "pipeline.seed_layers": "stage-local init is deterministic per module name",
    "zero_optimization.offload_optimizer": "optimizer state stays in HBM (288 GB per GPU)",
    "activation_checkpointing.partition_activations": "no tensor parallelism: nothing to partition",
    "activation_checkpointing.cpu_checkpointing": "checkpoints stay in HBM",
    "activation_checkpointing.contiguous_memory_optimization": "PyTorch caching allocator",
    "steps_per_print": "logging_steps / --log_every control logging",
    "wall_clock_breakdown": "phase timers are always on (timing_rank*.log)",
}
_MIFT_KEYS = {"kernels", "graph", "lmhead", "bucket_mb", "pp_partition", "pp_schedule", "micro_batch", "virtual_stages",
              "side_stream",
              "comm_timeout_s", "consistency_every", "max_inflight_steps", "strict"}


@dataclass
class MiftConfig:
    # --- DeepSpeed-compatible ---
    micro_batch_size: Optional[int] = None
    grad_accum: Optional[int] = None
    zero_stage: int = 1
    fp16: bool = False
    bf16: bool = False
    initial_scale_power: int = 16
    loss_scale_window: int = 1000
    lr: Optional[float] = None
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    gradient_clipping: float = 1.0
    activation_checkpointing: bool = False
    pp_stages: Optional[int] = None
    # --- mift.* (MI355X) ---
    kernels: bool = True
    graph: str = "auto"
    lmhead: str = "fused"
    bucket_mb: float = 25.0
    pp_partition: str = "balanced"
    pp_schedule: str = "1f1b"
    micro_batch: object = 0          # int, or "auto" (planner); 0 = the DeepSpeed micro-batch as is
    virtual_stages: object = None    # int, or "auto"; None = the app's default
    side_stream: Optional[bool] = None
    comm_timeout_s: Optional[int] = None
    consistency_every: int = 0
    max_inflight_steps: int = 2
    strict: bool = True
    # --- provenance ---
    source: Optional[str] = None
    found: bool = False
    no_effect: List[str] = field(default_factory=list)

    # ------------------------------------------------------------------
    @classmethod
    def from_dict(cls, d, source=None):
        c = cls(source=source, found=bool(d))
        m = d.get("mift", {}) or {}
        c.strict = bool(m.get("strict", True))
        unknown = [k for k in d if k not in _DS_KNOWN]
        unknown += [f"mift.{k}" for k in m if k not in _MIFT_KEYS]
        if unknown:
            msg = f"unknown config keys {unknown} in {source or 'config'}"
            if c.strict:
                raise ValueError(msg + " (set mift.strict=false to accept)")
            warnings.warn(msg)
        c.micro_batch_size = d.get("train_micro_batch_size_per_gpu")
        c.grad_accum = d.get("gradient_accumulation_steps")
        z = d.get("zero_optimization", {}) or {}
        c.zero_stage = int(z.get("stage", 1))
        if c.zero_stage not in (0, 1):
            raise ValueError(f"zero_optimization.stage {c.zero_stage} not supported (0 or 1)")
        f16 = d.get("fp16", {}) or {}
        c.fp16 = bool(f16.get("enabled", False))
        c.initial_scale_power = int(f16.get("initial_scale_power", 16))
        c.loss_scale_window = int(f16.get("loss_scale_window", 1000))
        c.bf16 = bool((d.get("bf16", {}) or {}).get("enabled", False))
        if c.fp16 and c.bf16:
            raise ValueError("fp16 and bf16 both enabled")
        opt = (d.get("optimizer", {}) or {}).get("params", {}) or {}
        c.lr = opt.get("lr")
        c.betas = tuple(opt.get("betas", (0.9, 0.999)))
        c.eps = float(opt.get("eps", 1e-8))
        c.weight_decay = float(opt.get("weight_decay", 0.0))
        c.gradient_clipping = float(d.get("gradient_clipping", 1.0))
        # DeepSpeed's section only configures deepspeed.checkpointing (never invoked by the reference,
        # SURVEY C20); recompute is requested explicitly (mift: "enabled": true, or the CLI flag)
        ac = d.get("activation_checkpointing", {}) or {}
        c.activation_checkpointing = bool(ac.get("enabled", False))
        pipe = d.get("pipeline", {}) or {}
        c.pp_stages = pipe.get("stages")
        if "partition_method" in pipe:
            pm = str(pipe["partition_method"]).lower()
            c.pp_partition = "uniform" if pm in ("uniform", "parameters") else "balanced"
        for path, why in _NO_EFFECT.items():
            sect, _, key = path.partition(".")
            hit = (key in (d.get(sect) or {})) if key else (sect in d)
            if hit:
                c.no_effect.append(f"{path}: {why}")
        c.kernels = bool(m.get("kernels", True))
        c.graph = str(m.get("graph", "auto"))
        c.lmhead = str(m.get("lmhead", "fused"))
        c.bucket_mb = float(m.get("bucket_mb", 25.0))
        c.pp_partition = str(m.get("pp_partition", c.pp_partition))
        c.pp_schedule = str(m.get("pp_schedule", "1f1b"))
        mb = m.get("micro_batch", 0)
        c.micro_batch = "auto" if str(mb).lower() == "auto" else int(mb)
        vs = m.get("virtual_stages")
        c.virtual_stages = None if vs is None else ("auto" if str(vs).lower() == "auto" else int(vs))
        c.side_stream = m.get("side_stream")
        c.comm_timeout_s = m.get("comm_timeout_s")
        c.consistency_every = int(m.get("consistency_every", 0))
        c.max_inflight_steps = int(m.get("max_inflight_steps", 2))
        for name, val, ok in [("graph", c.graph, ("auto", "on", "off")), ("lmhead", c.lmhead, ("fused", "blas")),
                              ("pp_partition", c.pp_partition, ("uniform", "balanced", "halves")),
                              ("pp_schedule", c.pp_schedule, ("1f1b",))]:
            if val not in ok:
                raise ValueError(f"mift.{name} must be one of {ok}, got {val!r}")
        return c

    @classmethod
    def from_json(cls, path):
        """Missing file -> defaults (the reference's inline fallback dict, `:179-199`)."""
        if path and os.path.isfile(path):
            with open(path) as f:
                return cls.from_dict(json.load(f), source=path)
        return cls(source=path)

    # ------------------------------------------------------------------
    def apply_env(self):
        """Export the process-wide toggles read by the runtime (explicit env vars win)."""
        os.environ.setdefault("MIFT_KERNELS", "1" if self.kernels else "0")
        os.environ.setdefault("MIFT_GRAPH", self.graph)
        os.environ.setdefault("MIFT_LMHEAD", self.lmhead)
        if self.side_stream is not None:
            os.environ.setdefault("MIFT_SIDE_STREAM", "1" if self.side_stream else "0")
        if self.comm_timeout_s:
            os.environ.setdefault("MIFT_COMM_TIMEOUT", str(int(self.comm_timeout_s)))

    def report(self):
        """Lines describing keys that were accepted without effect (logged by the apps)."""
        return [f"[config] accepted, no effect: {x}" for x in self.no_effect]

    def to_dict(self):
        return asdict(self)
