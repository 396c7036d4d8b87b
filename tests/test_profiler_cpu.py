"""--profile on the P1 app: a 2-rank gloo DDP run records a step window per rank
with the engine's named ranges, including one range per gradient bucket all-reduce."""
import json
import os

import pytest

from mift.utils import harness

BASE = ["--model", "gpt2-tiny", "--synthetic", "64", "--seq_len", "32", "--batch", "2", "--accum", "2",
        "--logging_steps", "0", "--step_log", "none", "--lr", "1e-2", "--no_save", "--run_name", "run"]


def _worker(rank, world, out):
    from mift.apps import ddp_finetune as app
    app.main(BASE + ["--out_root", out, "--logdir", os.path.join(out, "logs"), "--max_steps", "5",
                     "--profile", os.path.join(out, "prof"), "--profile_steps", "2:4"])
    return rank


def test_profile_window_per_rank(tmp_path):
    harness.run(_worker, 2, out=str(tmp_path))
    prof = tmp_path / "prof"
    for r in range(2):
        assert (prof / f"trace_rank{r}.json").stat().st_size > 0
        assert (prof / f"kernels_rank{r}.txt").stat().st_size > 0
        summ = json.loads((prof / f"ranges_rank{r}.json").read_text())
        assert summ["steps"] == [2, 4]
        rg = summ["ranges_ms"]
        assert rg["mift.step"]["n"] == 2            # exactly the two steps of the window
        assert rg["mift.optimizer"]["n"] == 2
        assert rg["mift.comm.grads"]["n"] == 2
        buckets = [k for k in rg if k.startswith("mift.comm.bucket")]
        assert buckets, rg                          # per-bucket all-reduce ranges
        trace = json.loads((prof / f"trace_rank{r}.json").read_text())
        names = {e.get("name") for e in trace.get("traceEvents", [])}
        assert "mift.step" in names and any(n and n.startswith("mift.comm.bucket") for n in names)


def test_parse_window():
    from mift.obs.profiler import parse_window
    assert parse_window("5:9") == (5, 9)
    assert parse_window("7") == (7, 10)
    assert parse_window("") == (3, 6)
    with pytest.raises(ValueError):
        parse_window("4:4")
