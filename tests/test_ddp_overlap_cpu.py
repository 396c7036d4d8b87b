"""DP engine behaviour on the CPU (gloo, 2 ranks):

* gradient buckets launch DURING backward (before the first layer's grads exist), not after;
* the per-step global label-token count comes from the shard plan (no per-step collective)
  and equals the count the old all-reduce produced;
* checkpoints without ``--run_name`` land in ONE directory chosen by rank 0, even when the
  ranks' clocks disagree (per-rank timestamps);
* the replica checksum is exact (bit patterns, not float sums).
"""
import os

import numpy as np
import torch

from mift.utils import harness

BASE = ["--model", "gpt2-tiny", "--synthetic", "64", "--seq_len", "32", "--batch", "2", "--accum", "2",
        "--logging_steps", "1", "--step_log", "none", "--lr", "1e-2"]


def _overlap_worker(rank, world):
    import torch.distributed as dist
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.parallel import dist as D
    from mift.train.trainer import TrainConfig, Trainer

    ctx = D.init(verbose=False, sanity=False)
    model = build_causal_lm("gpt2-tiny", seed=1)
    L.inject(model, L.LoraConfig(r=4, lora_alpha=8, target_modules=["c_attn", "c_proj"]), seed=1)
    ds = synthetic_openwebtext(16, 16, model.config.vocab_size, model.config.pad_token_id, seed=2)
    batcher = MicroBatcher(ds, 4, 1, rank=ctx.dp_rank, world=ctx.dp)  # one micro-step: no no_sync phase
    tr = Trainer(model, batcher, TrainConfig(batch=4, accum=1, precision="fp32", step_log="none", logging_steps=0,
                                             save_steps=0, bucket_mb=1e-4), ctx)
    events = []
    first = next(p for n, p in model.named_parameters() if "lora_A" in n)  # first module = last backward
    first.register_hook(lambda g: events.append("first_layer_grad"))
    real = dist.all_reduce

    def spy(t, *a, **k):
        events.append("all_reduce")
        return real(t, *a, **k)

    dist.all_reduce = spy
    try:
        mbs = next(iter(batcher.epoch(0)))
        tr.train_step(mbs)
    finally:
        dist.all_reduce = real
    log = list(tr.reducer.launch_log)
    D.destroy()
    return events, log, len(tr.reducer.buckets)


def test_buckets_launch_during_backward():
    res = harness.run(_overlap_worker, 2)
    for events, log, nb in res:
        assert nb > 2
        assert events.index("all_reduce") < events.index("first_layer_grad"), events
        assert sum(1 for _, w in log if w == "backward") >= nb - 1, log


def test_global_tokens_precomputed_from_shard_plan():
    """Each rank's precomputed count == the sum over ranks of the label tokens actually served
    (what the per-step all-reduce used to compute), for even and uneven (contiguous) shards."""
    from mift.data import MicroBatcher, synthetic_openwebtext
    ds = synthetic_openwebtext(37, 24, 500, 499, seed=7, full_length=False, mean_tokens=12)
    for mode in ("strided", "contiguous"):
        for world in (2, 3):
            per_rank = []
            for r in range(world):
                b = MicroBatcher(ds, 3, 2, rank=r, world=world, mode=mode, native=False)
                per_rank.append([(sum(int((mb["labels"][:, 1:] != -100).sum()) for mb in mbs), mbs.global_tokens)
                                 for mbs in b.epoch(0)])
            n = max(len(x) for x in per_rank)
            ref = [sum(x[s][0] for x in per_rank if s < len(x)) for s in range(n)]
            for x in per_rank:
                assert [g for _, g in x] == ref[:len(x)], (mode, world, x, ref)


def _noname_worker(rank, world, out):
    import datetime as _dt
    from mift.apps import ddp_finetune as app

    class _Clock:  # the two ranks' clocks straddle a second boundary
        class datetime:
            @staticmethod
            def now():
                return _dt.datetime(2026, 1, 1, 0, 0, 59 + rank) if rank == 0 else _dt.datetime(2026, 1, 1, 0, 1, 0)

    app.datetime = _Clock
    res = app.main(BASE + ["--out_root", out, "--logdir", os.path.join(out, "logs"), "--max_steps", "3",
                           "--save_steps", "1"])
    return res["save_dir"]


def test_checkpoint_dir_agreed_without_run_name(tmp_path):
    dirs = harness.run(_noname_worker, 2, out=str(tmp_path))
    assert dirs[0] == dirs[1]
    ck = os.path.join(dirs[0], "checkpoint-3")
    assert os.path.exists(os.path.join(ck, "optimizer.pt"))
    assert all(os.path.exists(os.path.join(ck, f"rng_state_{r}.pth")) for r in range(2))
    assert [d for d in os.listdir(str(tmp_path)) if d != "logs"] == [os.path.basename(dirs[0])]


def test_replica_checksum_is_exact():
    from mift.parallel.ddp import replica_checksum
    a = torch.randn(1000)
    b = a.clone()
    assert torch.equal(replica_checksum([a]), replica_checksum([b]))
    b[17] = torch.nextafter(b[17], torch.tensor(float("inf")))  # one ulp
    assert not torch.equal(replica_checksum([a]), replica_checksum([b]))
    c = a.clone()
    c[3], c[5] = a[5], a[3]  # same multiset, different positions: a float sum cannot see this
    assert not torch.equal(replica_checksum([a]), replica_checksum([c]))
    h = a.to(torch.bfloat16)
    assert replica_checksum([h]).shape == (1, 2)
    assert np.isfinite(replica_checksum([h]).numpy()).all()


def test_fused_claim_counts_each_tensor_once():
    """A tensor the fused forward claimed counts ONLY through the fused backward's notification:
    PyTorch also runs its post-accumulate-grad hook (the Functions take the LoRA tensors as inputs),
    and counting both launched the bucket half-way through backward — eager DP2 replicas diverged
    from step 1 on the GPU (tools/diag_ddp_eager.py, round 3).  Unclaimed tensors (eager path) still
    count through their hooks."""
    from mift import lora as L
    from mift.models import build_causal_lm
    from mift.parallel.ddp import GradReducer
    model = build_causal_lm("gpt2-tiny", seed=1)
    L.inject(model, L.LoraConfig(r=4, lora_alpha=8, target_modules=["c_attn", "c_proj"]), seed=1)
    arena = L.LoraArena(model)
    red = GradReducer(arena, world=2, bucket_mb=1e9)  # one bucket holding every tensor
    launches = []
    red._launch = lambda b, where="finish": (launches.append(where), b.__setitem__("launched", True))
    params = [p for _, p in arena.named]
    half = len(arena.offsets) // 2
    arena.grad_claim(arena.offsets[:half])  # the fused forward of the first half of the adapters
    for p in params:  # every hook fires (as PyTorch does for the fused inputs too)
        red._on_grad(p)
    assert launches == []  # the claimed half has not been reported yet
    arena.grad_ready(arena.offsets[:half - 1])
    assert launches == []
    arena.grad_ready(arena.offsets[half - 1:half])
    assert launches == ["backward"]
    red.finish = lambda: None
    red.remove()
    assert getattr(arena, "grad_claim", None) is None and getattr(arena, "grad_ready", None) is None
