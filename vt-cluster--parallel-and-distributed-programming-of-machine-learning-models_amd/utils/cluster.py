"""Cluster-side helpers: node audit, partition recommender, SSH helper.

Reference: ``utils/checker.py`` (sinfo/scontrol/uname/lscpu/free/df/ulimit
-> JSON), ``utils/Recommender.py`` (pick the partition with the most idle
CPUs from ``sinfo -N -o "%P %n %C %t"``, print an ``salloc`` line) and
``utils/Connect2Cluster.py`` (paramiko PTY shell from a ``.env``).

MI355X-first changes: the audit adds the GPU view (device count / names /
HBM per device from torch + ``rocm-smi``, xGMI link topology, RCCL/NCCL and
HSA environment, ROCm version), and the recommender ranks partitions by idle
GPUs (``%G`` gres, e.g. ``gpu:8``) and emits ``--gpus-per-node`` — the
reference filtered GPU partitions OUT because it targeted CPU nodes.
Every probe degrades to ``null`` when its tool is absent (no SLURM here).
"""
import json
import os
import platform
import re
import shutil
import subprocess


def run(cmd, timeout=20):
    if shutil.which(cmd[0]) is None:
        return None
    try:
        return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout).stdout.strip()
    except (subprocess.SubprocessError, OSError):
        return None


# ------------------------------------------------------------------ audit
def gpu_info():
    info = {"torch_visible": 0, "devices": []}
    try:
        import torch
        n = torch.cuda.device_count()
        info["torch_visible"] = n
        for i in range(n):
            p = torch.cuda.get_device_properties(i)
            info["devices"].append({"index": i, "name": p.name, "hbm_gib": round(p.total_memory / 2 ** 30, 1),
                                    "cus": p.multi_processor_count,
                                    "arch": getattr(p, "gcnArchName", None)})
    except Exception as e:  # noqa: BLE001 - a probe must not fail the audit
        info["error"] = str(e)
    info["rocm_smi_topology"] = run(["rocm-smi", "--showtopotype"])
    info["rocm_smi_memory"] = run(["rocm-smi", "--showmeminfo", "vram"])
    return info


def slurm_info():
    out = run(["sinfo", "-N", "-o", "%P %n %C %t %G"])
    if out is None:
        return None
    return {"sinfo": out.splitlines(), "config": run(["scontrol", "show", "config"])}


def os_info():
    lim = {}
    try:
        import resource
        for k in ("RLIMIT_NOFILE", "RLIMIT_NPROC", "RLIMIT_MEMLOCK", "RLIMIT_STACK"):
            lim[k] = resource.getrlimit(getattr(resource, k))
    except Exception:  # noqa: BLE001
        pass
    return {"uname": platform.uname()._asdict(), "python": platform.python_version(), "cpus": os.cpu_count(),
            "lscpu": run(["lscpu"]), "free": run(["free", "-g"]), "df": run(["df", "-h", "."]), "limits": lim,
            "rocm_version": _read("/opt/rocm/.info/version")}


def _read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError:
        return None


def comm_env():
    keys = [k for k in os.environ if k.startswith(("NCCL_", "RCCL_", "HSA_", "HIP_", "GLOO_", "MASTER_", "TORCH_NCCL",
                                                  "OMP_NUM_THREADS", "SLURM_JOB"))]
    return {k: os.environ[k] for k in sorted(keys)}


def audit():
    try:
        import torch
        tv = torch.__version__
    except Exception:  # noqa: BLE001
        tv = None
    return {"host": platform.node(), "torch": tv, "os": os_info(), "gpu": gpu_info(), "slurm": slurm_info(),
            "comm_env": comm_env()}


# ------------------------------------------------------------------ recommender
def parse_sinfo(lines):
    """``sinfo -N -o "%P %n %C %t [%G]"`` lines -> {partition: [{node, idle, total, gpus}]} (down nodes dropped)."""
    parts = {}
    for ln in lines:
        f = ln.split()
        if len(f) < 4 or f[0] == "PARTITION":
            continue
        part, node, cpus, state = f[0].strip("*").lower(), f[1], f[2], f[3].lower()
        try:
            _, idle, _, total = map(int, cpus.split("/"))
        except ValueError:
            continue
        if "down" in state or "drain" in state:
            continue
        gpus = 0
        if len(f) > 4:
            m = re.search(r"gpu(?::[\w-]+)?:(\d+)", f[4])
            gpus = int(m.group(1)) if m else 0
        if state.startswith(("alloc", "mix")) and gpus:
            gpus = 0 if state.startswith("alloc") else gpus  # a mixed node may still have free GPUs
        parts.setdefault(part, []).append({"node": node, "idle": idle, "total": total, "gpus": gpus,
                                           "state": state})
    return parts


def recommend(parts, max_nodes=8, prefer_gpu=True):
    """-> (partition, [nodes]) maximising idle GPUs (then idle CPUs); None if nothing is free."""
    if not parts:
        return None

    def score(kv):
        nodes = [n for n in kv[1] if n["idle"] > 0 or n["gpus"] > 0]
        return (sum(n["gpus"] for n in nodes) if prefer_gpu else 0, sum(n["idle"] for n in nodes))

    best = max(parts.items(), key=score)
    nodes = [n for n in best[1] if (n["gpus"] > 0 if prefer_gpu and score(best)[0] else n["idle"] > 0)]
    if not nodes:
        return None
    return best[0], nodes[:max_nodes]


def salloc_cmd(partition, nodes=1, gpus_per_node=8, cpus_per_task=16, time="01:00:00", nodelist=None):
    cmd = (f"salloc --partition={partition} --nodes={nodes} --ntasks-per-node=1 --gpus-per-node={gpus_per_node} "
           f"--cpus-per-task={cpus_per_task} --time={time}")
    if nodelist:
        cmd += " --nodelist=" + ",".join(nodelist)
    return cmd


# ------------------------------------------------------------------ ssh
def load_env(path=".env"):
    env = {}
    if os.path.exists(path):
        with open(path) as f:
            for ln in f:
                ln = ln.strip()
                if ln and not ln.startswith("#") and "=" in ln:
                    k, v = ln.split("=", 1)
                    env[k.strip()] = v.strip().strip('"').strip("'")
    return env


def ssh_command(env):
    host, user = env.get("HOST") or os.getenv("HOST"), env.get("USER") or os.getenv("USER")
    if not host or not user:
        raise SystemExit("Please set HOST and USER in environment or .env file.")
    port = env.get("PORT", os.getenv("PORT", "22"))
    keep = env.get("KEEPALIVE", os.getenv("KEEPALIVE", "60"))
    return ["ssh", "-tt", "-p", str(port), "-o", f"ServerAliveInterval={keep}", f"{user}@{host}"]


def connect(env_path=".env"):
    """Interactive login shell on the cluster head node (system ssh; the PTY, SIGWINCH and
    Ctrl-C forwarding the reference re-implemented with paramiko come with it)."""
    cmd = ssh_command(load_env(env_path))
    return subprocess.call(cmd)


def main_checker(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="Cluster / node audit (MI355X)")
    ap.add_argument("--output", "-o", help="write JSON here")
    a = ap.parse_args(argv)
    rep = audit()
    s = json.dumps(rep, indent=2, default=str)
    if a.output:
        with open(a.output, "w") as f:
            f.write(s)
        print(f"✅ wrote {a.output}")
    else:
        print(s)
    return rep


def main_recommender(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="Recommend a partition + salloc line")
    ap.add_argument("--max_nodes", type=int, default=8)
    ap.add_argument("--cpu", action="store_true", help="rank by idle CPUs (reference behaviour)")
    ap.add_argument("--sinfo_file", default=None, help="parse saved sinfo output instead of running sinfo")
    a = ap.parse_args(argv)
    if a.sinfo_file:
        with open(a.sinfo_file) as f:
            lines = f.read().splitlines()
    else:
        out = run(["sinfo", "-N", "-o", "%P %n %C %t %G"])
        if out is None:
            print("❌ sinfo not available on this host")
            return None
        lines = out.splitlines()
    rec = recommend(parse_sinfo(lines), a.max_nodes, prefer_gpu=not a.cpu)
    if rec is None:
        print("❌ No partition with free resources found.")
        return None
    part, nodes = rec
    gpn = max((n["gpus"] for n in nodes), default=0)
    print(f"✅ partition={part} nodes={[n['node'] for n in nodes]}")
    print(salloc_cmd(part, len(nodes), gpn or 0, nodelist=[n["node"] for n in nodes]))
    return rec
