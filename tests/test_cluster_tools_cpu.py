"""Cluster tools: sinfo parsing / partition recommendation, salloc line, audit JSON, ssh command."""
import json

from mift.utils import cluster as CL

SINFO = """PARTITION NODELIST CPUS(A/I/O/T) STATE GRES
torch* hpc01 0/8/0/8 idle (null)
torch* hpc02 8/0/0/8 alloc (null)
mi355x gpu01 0/128/0/128 idle gpu:8
mi355x gpu02 64/64/0/128 mix gpu:mi355x:8
mi355x gpu03 0/128/0/128 down gpu:8
debug dbg01 0/4/0/4 idle (null)"""


def test_parse_and_recommend():
    parts = CL.parse_sinfo(SINFO.splitlines())
    assert set(parts) == {"torch", "mi355x", "debug"}
    assert [n["node"] for n in parts["mi355x"]] == ["gpu01", "gpu02"]   # down node dropped
    part, nodes = CL.recommend(parts)
    assert part == "mi355x" and nodes[0]["gpus"] == 8
    cpu_part, _ = CL.recommend(parts, prefer_gpu=False)
    assert cpu_part == "mi355x"          # most idle CPUs too
    cmd = CL.salloc_cmd(part, 2, 8, nodelist=["gpu01", "gpu02"])
    assert "--gpus-per-node=8" in cmd and "--nodelist=gpu01,gpu02" in cmd


def test_audit_is_json_serialisable():
    rep = CL.audit()
    s = json.dumps(rep, default=str)
    assert "gpu" in rep and "os" in rep and rep["os"]["cpus"] >= 1 and len(s) > 100


def test_ssh_command(tmp_path):
    env = tmp_path / ".env"
    env.write_text("HOST=head.example\nUSER=alice\nPORT=2222\nKEEPALIVE=30\n")
    cmd = CL.ssh_command(CL.load_env(str(env)))
    assert cmd[-1] == "alice@head.example" and "2222" in cmd and "ServerAliveInterval=30" in cmd
