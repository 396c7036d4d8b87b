"""Bring-up env mapping (torchrun / SLURM fallbacks) and the parallel_utils compat shim."""
import os
import subprocess
import sys

from mift.parallel.dist import _first_slurm_host, env_rank_info

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_env_rank_info(monkeypatch):
    for k in ["RANK", "WORLD_SIZE", "LOCAL_RANK", "SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID"]:
        monkeypatch.delenv(k, raising=False)
    assert env_rank_info() == (0, 1, 0)
    monkeypatch.setenv("SLURM_PROCID", "5")
    monkeypatch.setenv("SLURM_NTASKS", "8")
    monkeypatch.setenv("SLURM_LOCALID", "1")
    assert env_rank_info() == (5, 8, 1)          # B6: RANK falls back to SLURM_PROCID too
    monkeypatch.setenv("RANK", "2")
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert env_rank_info()[:2] == (2, 4)


def test_slurm_nodelist(monkeypatch):
    monkeypatch.setenv("SLURM_JOB_NODELIST", "hpc[12-15,20],gpu3")
    assert _first_slurm_host() == "hpc12"
    monkeypatch.setenv("SLURM_JOB_NODELIST", "node7")
    assert _first_slurm_host() == "node7"


def test_parallel_utils_single_process():
    code = ("import sys; sys.path.insert(0, %r); from utils.parallel_utils import *; "
            "init_distributed(0); print(world_size(), is_main_process())" % ROOT)
    env = dict(os.environ, MIFT_DEVICE="cpu", MASTER_ADDR="127.0.0.1", MASTER_PORT="29677", WORLD_SIZE="1")
    env.pop("RANK", None)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "1 True"
