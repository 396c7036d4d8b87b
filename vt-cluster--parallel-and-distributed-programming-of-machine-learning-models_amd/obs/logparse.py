"""Log evaluation and timing summaries over the reference line formats.

Equivalent of the reference's aggregators:
  * ``evaluate_logs`` — the ``labs/tiny/eval_logs.py`` report: rendezvous
    uniqueness, rank coverage 0..W-1, per-node version drift, preflight
    visibility, step-time / throughput P50/P95, TRAIN_RUNTIME_SEC, eval and
    INFER global lines, failure signatures, PASS/CHECK verdict;
  * ``training_seconds`` / ``summarize_times`` — ``summarize_*_times.py``:
    max ``[Training] x sec`` over ``timing_rank*.log`` + meta + wall clock;
  * ``scaling`` — S(n) = T(1)/T(n), E(n) = S(n)/n (explanation/cluster_lab_LatestLab.pdf p.2).
Our own logs emit these formats verbatim (mift.obs.timing), so one parser
reads both frameworks' runs.
"""
import glob
import json
import os
import re
from collections import Counter

PATTERNS = {
    "rank": re.compile(r"\[RANK\s+(\d+)\]\s+WORLD_SIZE=(\d+)"),
    "rdzv": re.compile(r"torchrun:\s+nnodes=(\d+)\s+nproc_per_node=(\d+)\s+node_rank=(\d+)\s+rdzv=(\S+)"),
    "sanity": re.compile(r"NODE\s+(\S+)\s+OK\s+->\s+PY\s+(\S+)\s+torch\s+(\S+)\s+tfm\s+(\S+)\s+numpy\s+(\S+)"
                         r"\s+datasets\s+(\S+)\s+root\s+(\S+)"),
    "fail": re.compile(r"(Traceback|ERROR|RuntimeError|OSError|Address already in use|Timed out)", re.I),
    "step": re.compile(r"\[rank\s+(\d+)\s+\|\s+step\s+(\d+)\]\s+.*?step_ms=([\d.]+)\s+samples_per_sec=([\d.]+)"
                       r"\s+tokens_per_sec=([\d.]+)"),
    "runtime": re.compile(r"TRAIN_RUNTIME_SEC=([\d.]+)"),
    "eval": re.compile(r"(?:eval_accuracy|EVAL accuracy)=\s*([0-9]*\.?[0-9]+)"),
    "infer": re.compile(r"\[RANK 0\]\s+INFER.*global_accuracy=\s*([0-9]*\.?[0-9]+|NA).*?"
                        r"global_samples_per_sec=([\d.]+).*?global_tokens_per_sec=([\d.]+)", re.S),
    "p1_step": re.compile(r"rank=(\d+) step (\d+) ([\d.]+)s"),
    "p2_loss": re.compile(r"\[R(\d+)\] ep=(\d+) step=(\d+) loss=([\d.]+)"),
    "training": re.compile(r"\[Training\]\s+([\d.]+)\s+sec"),
}


def percentile(vals, q):
    if not vals:
        return None
    s = sorted(float(x) for x in vals)
    k = (len(s) - 1) * q
    f = int(k)
    c = min(f + 1, len(s) - 1)
    return s[f] if f == c else s[f] + (s[c] - s[f]) * (k - f)


def _read(p):
    try:
        with open(p, "r", errors="replace") as f:
            return f.read()
    except OSError as e:
        return f"[[could not read {p}: {e}]]"


def read_preflight(path):
    st = {}
    if not path or not os.path.exists(path):
        return st
    for line in _read(path).splitlines():
        parts = line.split()
        if not parts:
            continue
        kv = dict(p.split("=", 1) for p in parts[1:] if "=" in p)
        st[parts[0]] = (kv.get("proj", "missing"), kv.get("pkgs", "missing"))
    return st


def evaluate_logs(paths, preflight=None):
    r = {"ranks": set(), "ws": Counter(), "rdzv": [], "sanity": {}, "fail": [], "fail_files": Counter(),
         "step_ms": [], "sps": [], "tps": [], "runtime": [], "eval": [], "infer": [], "p1_steps": [],
         "p2_loss": []}
    for p in paths:
        txt = _read(p)
        for m in PATTERNS["rank"].finditer(txt):
            r["ranks"].add(int(m.group(1)))
            r["ws"][int(m.group(2))] += 1
        r["rdzv"] += [(int(a), int(b), int(c), d) for a, b, c, d in PATTERNS["rdzv"].findall(txt)]
        for m in PATTERNS["sanity"].finditer(txt):
            r["sanity"][m.group(1)] = m.groups()[1:]
        for m in PATTERNS["step"].finditer(txt):
            r["step_ms"].append(float(m.group(3)))
            r["sps"].append(float(m.group(4)))
            r["tps"].append(float(m.group(5)))
        r["runtime"] += [float(x) for x in PATTERNS["runtime"].findall(txt)]
        r["eval"] += [float(x) for x in PATTERNS["eval"].findall(txt)]
        r["infer"] += [m.groups() for m in PATTERNS["infer"].finditer(txt)]
        r["p1_steps"] += [float(x[2]) for x in PATTERNS["p1_step"].findall(txt)]
        r["p2_loss"] += [float(x[3]) for x in PATTERNS["p2_loss"].findall(txt)]
        hits = [m.group(0) for m in PATTERNS["fail"].finditer(txt)]
        if hits:
            r["fail_files"][os.path.basename(p)] = len(hits)
            r["fail"] += [f"{os.path.basename(p)}: {h}" for h in hits]
    r["preflight"] = read_preflight(preflight)
    uniq = sorted({(a, b, d) for a, b, _, d in r["rdzv"]})
    ok = bool(uniq) and bool(r["ranks"]) and len(r["ws"]) == 1
    if ok:
        ws = next(iter(r["ws"]))
        ok = not (set(range(ws)) - r["ranks"]) and not r["fail"]
    r["rdzv_unique"], r["verdict"] = uniq, ok
    return r


def format_report(r, job="?"):
    L = ["=" * 72, f" EVALUATION REPORT FOR JOB {job}", "=" * 72, "", "[RDZV] Rendezvous records (unique):"]
    L += [f"  - nnodes={a}  nproc_per_node={b}  endpoint={d}" for a, b, d in r["rdzv_unique"]] or \
        ["  (!) No rendezvous banner found."]
    if len(r["rdzv_unique"]) > 1:
        L.append("  (!) Inconsistent rendezvous configs detected.")
    if r["ranks"]:
        L += ["", "[RANKS] Rank coverage:",
              f"  - ranks seen: min={min(r['ranks'])}  max={max(r['ranks'])}  count={len(r['ranks'])}",
              f"  - WORLD_SIZE candidates (value -> observations): {sorted(r['ws'].items())}"]
        if len(r["ws"]) == 1:
            ws = next(iter(r["ws"]))
            miss = sorted(set(range(ws)) - r["ranks"])
            L.append(f"  (!) Missing ranks: {miss[:15]}" if miss else "  ✓ All ranks accounted for (max == WORLD_SIZE-1).")
        else:
            L.append("  (!) Multiple WORLD_SIZE values observed; check consistency.")
    else:
        L += ["", "[RANKS] (!) No '[RANK r] WORLD_SIZE=w' lines found."]
    if r["sanity"]:
        L += ["", "[SANITY] Per-node versions:"]
        for h, v in sorted(r["sanity"].items()):
            L.append(f"  {h:<16} " + " ".join(f"{x:<8}" for x in v))
        for name, i in [("PY", 0), ("torch", 1), ("tfm", 2), ("numpy", 3), ("datasets", 4)]:
            vals = Counter(v[i] for v in r["sanity"].values())
            if len(vals) > 1:
                L.append(f"  (!) Version drift in {name}: {dict(vals)}")
    if r["preflight"]:
        ok = sum(1 for v in r["preflight"].values() if v == ("ok", "ok"))
        L += ["", "[PREFLIGHT] Project/pkgs visibility by node:"]
        L += [f"  {h:<16} proj={p:<7} pkgs={k:<7}" for h, (p, k) in sorted(r["preflight"].items())]
        L.append(f"  Summary: {ok}/{len(r['preflight'])} nodes had both proj & pkgs visible.")
    if r["step_ms"]:
        L += ["", "[THROUGHPUT] Step-time & throughput (all ranks, across steps):",
              f"  - step_ms:     P50={percentile(r['step_ms'], .5):.2f}  P95={percentile(r['step_ms'], .95):.2f}",
              f"  - samples/sec: P50={percentile(r['sps'], .5):.1f} P95={percentile(r['sps'], .95):.1f}",
              f"  - tokens/sec:  P50={percentile(r['tps'], .5):.1f} P95={percentile(r['tps'], .95):.1f}"]
    if r["p1_steps"]:
        L.append(f"  - P1 step s:  P50={percentile(r['p1_steps'], .5):.3f}  P95={percentile(r['p1_steps'], .95):.3f}")
    if r["runtime"]:
        L.append(f"  - TRAIN_RUNTIME_SEC (rank0): min={min(r['runtime']):.2f} max={max(r['runtime']):.2f}")
    if r["eval"]:
        L += ["", f"[EVAL] eval_accuracy (epoch logs): best={max(r['eval']):.4f} last={r['eval'][-1]:.4f}"]
    if r["infer"]:
        a, s, t = r["infer"][-1]
        L.append(f"[INFER] global_accuracy={a} global_samples_per_sec={float(s):.1f} global_tokens_per_sec={float(t):.1f}")
    if r["p2_loss"]:
        L.append(f"[P2] loss first={r['p2_loss'][0]:.4f} last={r['p2_loss'][-1]:.4f} ({len(r['p2_loss'])} lines)")
    if r["fail"]:
        L += ["", "[FAILURES] Signatures found:"]
        L += [f"  - {f}: {c} hits" for f, c in r["fail_files"].most_common(5)]
        L += [f"    e.g., {x}" for x in r["fail"][:8]]
    else:
        L += ["", "[FAILURES] ✓ No failure signatures detected."]
    L += ["", "[VERDICT]", "  ✓ PASS" if r["verdict"] else "  ✗ CHECK LOGS (see sections above)"]
    return "\n".join(L)


# ---------------------------------------------------------------- timings
def training_seconds(logdir):
    secs = []
    for p in glob.glob(os.path.join(logdir, "timing_rank*.log")):
        secs += [float(x) for x in PATTERNS["training"].findall(_read(p))]
    return max(secs) if secs else float("nan")


def read_meta(logdir):
    for name in ("meta.final.json", "meta.json", "run_meta.json"):
        mp = os.path.join(logdir, name)
        if os.path.exists(mp):
            try:
                with open(mp) as f:
                    return json.load(f)
            except (OSError, ValueError):
                pass
    return {}


def read_wall(logdir):
    wp = os.path.join(logdir, "wallclock_seconds.txt")
    try:
        with open(wp) as f:
            return int(float(f.read().strip()))
    except (OSError, ValueError):
        return None


def summarize_times(logdirs, title):
    out = [title, "-" * 70]
    for ld in logdirs:
        meta, t, wall = read_meta(ld), training_seconds(ld), read_wall(ld)
        # N = ranks (GPUs) when known: the reference's N was nodes with one rank each
        n = meta.get("world_size", meta.get("n_gpus", meta.get("nnodes", "?")))
        label = f"N={n!s:>2}  dataset={meta.get('dataset', '?')!s:>6}  job={meta.get('job_id', os.path.basename(ld))}"
        right = f"train={t:.2f}s" if t == t else "train=NA"
        if wall is not None:
            right += f"  wall={wall}s"
        out.append(f"{label:<40} {right}")
    return "\n".join(out)


def scaling(times_by_n):
    """{n: seconds} -> {n: (speedup S(n)=T(1)/T(n), efficiency E(n)=S(n)/n)}."""
    t1 = times_by_n.get(1)
    if not t1:
        return {}
    return {n: (t1 / t, t1 / t / n) for n, t in sorted(times_by_n.items()) if t}
