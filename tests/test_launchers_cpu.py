"""Launcher / environment scripts: syntax, sanity banner, ACTION dispatch through the
multi-node launcher's local (no-SLURM) path with a real torchrun rendezvous on 127.0.0.1."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("script", sorted(glob.glob(os.path.join(ROOT, "scripts", "*.sh"))
                                          + glob.glob(os.path.join(ROOT, "scripts", "*.sbatch"))))
def test_shell_syntax(script):
    subprocess.run(["bash", "-n", script], check=True)


def test_sanity_line_parses():
    from mift.apps import run_action
    from mift.obs import logparse
    line = run_action.sanity_line()
    assert logparse.PATTERNS["sanity"].search(line) if hasattr(logparse, "PATTERNS") else "OK -> PY" in line


def test_unknown_action():
    from mift.apps import run_action
    with pytest.raises(SystemExit):
        run_action.resolve("nope")


def test_env_script_probe():
    out = subprocess.run(["bash", "-c", f"source {ROOT}/scripts/env_mi355x.sh && echo HF=$HF_HUB_OFFLINE"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "[env] torch" in out.stdout and "HF=1" in out.stdout


def test_launch_tiny_write(tmp_path):
    dst = tmp_path / "launch_tiny.sh"
    subprocess.run(["bash", f"{ROOT}/scripts/launch_tiny.sh", "--write", str(dst)], check=True)
    txt = dst.read_text()
    assert f'ROOT="{ROOT}"' in txt
    subprocess.run(["bash", "-n", str(dst)], check=True)


def test_launch_tiny_local_eval(tmp_path):
    """ACTION=eval through launcher -> torchrun (1 rank) -> run_action -> labs/tiny/eval_logs.py."""
    log = tmp_path / "train.77.0.out"
    log.write_text("torchrun: nnodes=1 nproc_per_node=2 node_rank=0 rdzv=127.0.0.1:29500\n"
                   "[RANK 0] WORLD_SIZE=2\n[RANK 1] WORLD_SIZE=2\n"
                   "[rank 0 | step 10] step_ms=12.5 samples_per_sec=640.0 tokens_per_sec=81920.0\n"
                   "TRAIN_RUNTIME_SEC=3.2\nEVAL accuracy=0.41\n")
    env = dict(os.environ, ACTION="eval", GPUS_PER_NODE="1", MASTER_PORT="29717")
    env.pop("SLURM_JOB_ID", None)
    out = subprocess.run(["bash", f"{ROOT}/scripts/launch_tiny.sh", "--job", "77", "--logs-dir", str(tmp_path)],
                         capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "torchrun: nnodes=1 nproc_per_node=1 node_rank=0" in out.stdout
    assert "NODE " in out.stdout and "EVALUATION REPORT" in out.stdout
