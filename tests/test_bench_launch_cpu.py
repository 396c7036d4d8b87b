"""bench.py forms the world it is asked for, or fails (VERDICT r3 "Next round" #1).

`python bench.py --gpus N` with no torchrun environment starts the N ranks itself (a child
torch.distributed.run), and the JSON line reports the world that actually ran; a mismatch between
--gpus and the launched world, or a request no launcher can satisfy, exits non-zero instead of
measuring something else.  CPU / gloo here; the GPU box runs the same code over RCCL."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--steps", "1", "--warmup", "0", "--epoch_lines", "0"]


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                        "MASTER_ADDR", "MASTER_PORT", "MIFT_BACKEND")}
    e.update(OMP_NUM_THREADS="2", **kw)
    return e


def _run(args, env=None, timeout=600):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env or _env(), cwd=ROOT)


def _json(out):
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout + out.stderr[-3000:]
    return json.loads(lines[0])


def test_bench_launches_two_ranks_itself():
    out = _run(["--gpus", "2", "--accum", "2", "--seq_len", "32"] + SMALL)
    assert out.returncode == 0, out.stderr[-3000:]
    r = _json(out)
    assert r["n_gpus"] == 2
    assert r["config"]["parallelism"] == "dp2"
    assert r["config"]["global_batch"] == 4 and r["config"]["config_id"] == 2
    assert r["value"] > 0 and r["steps"] == 1


def test_bench_config3_pipeline_grid():
    # BASELINE config #3 on 4 ranks (tiny OPT so it fits a CPU test): a dp1 x pp4 grid, auto micro-batch
    out = _run(["--gpus", "4", "--config", "3", "--model", "opt-tiny", "--precision", "fp32", "--seq_len", "32",
                "--accum", "8"] + SMALL)
    assert out.returncode == 0, out.stderr[-3000:]
    r = _json(out)
    assert r["n_gpus"] == 4 and r["config"]["parallelism"] == "dp1xpp4"
    assert r["config"]["config_id"] == 3
    plan = r["config"]["micro_batch_plan"]
    assert plan is not None and 8 % plan["micro_batch"] == 0


def test_bench_world_mismatch_fails():
    # torchrun-style env with a different world than requested: must not silently measure 1 rank
    out = _run(["--gpus", "2"] + SMALL, env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
                                               MASTER_ADDR="127.0.0.1", MASTER_PORT="29731"))
    assert out.returncode != 0 and out.stdout.strip() == ""
    assert "WORLD_SIZE=1" in out.stderr


def test_bench_no_gpu_fails_loudly():
    # the default (GPU) path with no GPU visible: no CPU downgrade, no JSON line
    out = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert out.returncode != 0 and out.stdout.strip() == ""
    assert "GPU" in out.stderr


def test_bench_bad_pipeline_grid_fails():
    out = _run(["--gpus", "2", "--config", "3"] + SMALL)
    assert out.returncode != 0 and "pipeline stages" in out.stderr


def test_bench_interleaved_pipeline_grid():
    """--virtual_stages 2: two model chunks per pipeline rank (interleaved 1F1B over the wrap-around link)."""
    out = _run(["--gpus", "2", "--config", "3", "--pp", "2", "--virtual_stages", "2", "--micro_batch", "2",
                "--model", "opt-tiny", "--precision", "fp32", "--seq_len", "32", "--accum", "4"] + SMALL)
    assert out.returncode == 0, out.stderr[-3000:]
    r = _json(out)
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp1xpp2xv2"
    # OPT pipelines default to half-layer partition units (the head's cost moves half layers off the last chunk)
    sp = r["config"]["split"]
    assert len(sp) == 4 and sum(sp) == 4 and all(2 * x == int(2 * x) for x in sp) and r["value"] > 0


def test_bench_config3_reports_epoch():
    """The OPT half of the BASELINE metric: config 3 reports wall-clock/epoch (fresh model + Trainer over
    the medium-shaped corpus, timed from its first step) like config 2 (VERDICT r4 missing #2)."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.parse_args(["--config", "3"]).epoch_lines == 20000
    assert bench.parse_args(["--config", "2"]).epoch_lines == 20000
    args = ["--gpus", "2", "--config", "3", "--pp", "2", "--model", "opt-tiny", "--precision", "fp32", "--seq_len",
            "32", "--accum", "4", "--device", "cpu", "--steps", "1", "--warmup", "0", "--epoch_lines", "16"]
    out = _run(args)
    assert out.returncode == 0, out.stderr[-3000:]
    r = _json(out)
    assert r["wall_clock_epoch_s"] is not None and r["wall_clock_epoch_s"] > 0
    assert r["epoch"]["lines"] == 16 and r["epoch"]["steps"] == 4  # 16 lines / (1 x 4 per step)
    assert r["config"]["parallelism"].startswith("dp1xpp2")
