"""Failure detection / recovery: injected faults tear the job down with a non-zero exit,
a hung rank is caught by the collective timeout, and --resume auto continues bit-exactly."""
import os
import subprocess
import sys

import pytest
import torch

from mift.utils import harness

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "scripts", "finetune_lora_distilgpt2.py")
BASE = ["--model", "gpt2-tiny", "--synthetic", "64", "--seq_len", "32", "--batch", "2", "--accum", "2",
        "--logging_steps", "1", "--step_log", "none", "--lr", "1e-2"]


def _torchrun(args, env_extra, timeout=240):
    port = str(harness.free_port())
    env = dict(os.environ, MIFT_DEVICE="cpu", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", port, SCRIPT] + args
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("kind", ["exit", "raise"])
def test_fault_tears_down_job(tmp_path, kind):
    r = _torchrun(BASE + ["--out_root", str(tmp_path), "--logdir", str(tmp_path / "logs"), "--max_steps", "6"],
                  {"MIFT_FAULT": f"1:2:{kind}"})
    assert r.returncode != 0
    assert "[FAULT] injecting" in r.stdout + r.stderr


def test_hang_caught_by_collective_timeout(tmp_path):
    r = _torchrun(BASE + ["--out_root", str(tmp_path), "--logdir", str(tmp_path / "logs"), "--max_steps", "6"],
                  {"MIFT_FAULT": "1:2:hang:micro", "GLOO_SOCKET_TIMEOUT": "6", "MIFT_FAULT_HANG_S": "15"})
    assert r.returncode != 0
    assert "Timed out" in r.stdout + r.stderr  # the healthy rank's collective timeout fired first


def _run(rank, world, out, extra):
    from mift.apps.ddp_finetune import main
    res = main(BASE + ["--out_root", out, "--logdir", os.path.join(out, "logs"), "--run_name", "run"] + extra)
    from mift import lora as L  # noqa: F401
    return res


def _adapter(out):
    from safetensors.torch import load_file
    return load_file(os.path.join(out, "run", "adapter_model.safetensors"))


def test_resume_auto_is_exact(tmp_path):
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    harness.run(_run, 2, out=a, extra=["--max_steps", "5"])
    with pytest.raises(RuntimeError):
        harness.run(_run, 2, out=b, extra=["--max_steps", "5", "--save_steps", "1"], env={"MIFT_FAULT": "*:3:raise"})
    assert os.path.isdir(os.path.join(b, "run", "checkpoint-2"))
    harness.run(_run, 2, out=b, extra=["--max_steps", "5", "--save_steps", "1", "--resume", "auto"])
    sa, sb = _adapter(a), _adapter(b)
    assert sa.keys() == sb.keys()
    for k in sa:
        torch.testing.assert_close(sa[k], sb[k], atol=1e-6, rtol=1e-5)


def _diverge_worker(rank, world):
    import torch
    from mift import lora as L
    from mift.data import MicroBatcher, synthetic_openwebtext
    from mift.models import build_causal_lm
    from mift.parallel import dist as D
    from mift.train.trainer import TrainConfig, Trainer

    ctx = D.init(verbose=False, sanity=False)
    model = build_causal_lm("opt-tiny", seed=3)
    if rank == 1:  # a replica that loaded different weights
        with torch.no_grad():
            next(p for p in model.parameters()).add_(0.5)
    L.inject(model, L.LoraConfig(r=4, lora_alpha=8, target_modules=["q_proj", "v_proj"]), seed=3)
    ds = synthetic_openwebtext(16, 8, model.config.vocab_size, model.config.pad_token_id, seed=5)
    try:
        Trainer(model, MicroBatcher(ds, 2, 2, rank=ctx.dp_rank, world=ctx.dp),
                TrainConfig(precision="fp32", step_log="none", logging_steps=0, save_steps=0), ctx)
        return "no-error"
    except RuntimeError as e:
        return "diverged" if "replica divergence" in str(e) else repr(e)
    finally:
        D.destroy()


def test_replica_divergence_detected():
    """DP replicas are not broadcast at start (identical init by seed); a checksum all-reduce
    over the DP group must catch a replica whose weights differ."""
    assert harness.run(_diverge_worker, 2) == ["diverged", "diverged"]
