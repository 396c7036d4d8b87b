"""Log-format conformance: our emitters feed the reference-format parsers."""
import os

from mift.obs import timing as T
from mift.obs.logparse import evaluate_logs, format_report, scaling, summarize_times, training_seconds
from mift.obs.tb import SummaryWriter, read_events


def test_eval_logs_pass(tmp_path):
    lines = ["torchrun: nnodes=1 nproc_per_node=2 node_rank=0 rdzv=127.0.0.1:29500",
             "[RANK 0] WORLD_SIZE=2", "[RANK 1] WORLD_SIZE=2",
             T.lab_step_line(0, 1, 12.5, 100.0, 12800.0), T.lab_step_line(1, 1, 13.5, 90.0, 11520.0),
             "[RANK 0] TRAIN_RUNTIME_SEC=3.210", "[RANK 0] EVAL accuracy=0.8123",
             "[RANK 0] INFER global_accuracy=0.8000 global_samples_per_sec=1234.5 global_tokens_per_sec=158016.0",
             T.p2_loss_line(3, 0, 10, 2.3456, 1.2)]
    p = tmp_path / "train.77.0.out"
    p.write_text("\n".join(lines) + "\n")
    r = evaluate_logs([str(p)])
    assert r["verdict"] and r["ranks"] == {0, 1} and r["eval"] == [0.8123] and r["p2_loss"] == [2.3456]
    rep = format_report(r, "77")
    assert "✓ PASS" in rep and "P50=13.00" in rep
    bad = tmp_path / "train.78.0.out"
    bad.write_text("[RANK 0] WORLD_SIZE=2\nTraceback (most recent call last):\n")
    assert not evaluate_logs([str(bad)])["verdict"]


def test_timing_summary(tmp_path):
    for r, s in [(0, 10.0), (1, 12.5)]:
        lg = T.PhaseLogger(str(tmp_path), r)
        lg.log("Training", s, echo=False)
    (tmp_path / "wallclock_seconds.txt").write_text("20\n")
    assert training_seconds(str(tmp_path)) == 12.5
    assert "train=12.50s  wall=20s" in summarize_times([str(tmp_path)], "t")
    s = scaling({1: 8.0, 2: 4.2, 4: 2.5})
    assert abs(s[2][0] - 8 / 4.2) < 1e-9 and abs(s[4][1] - 0.8) < 1e-9


def test_tensorboard_roundtrip(tmp_path):
    w = SummaryWriter(str(tmp_path))
    w.add_scalar("loss", 1.5, 3)
    w.add_scalar("acc", 0.25, 4)
    w.close()
    ev = read_events(w.path)
    assert ev == [(3, {"loss": 1.5}), (4, {"acc": 0.25})]
