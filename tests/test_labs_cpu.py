"""Remaining labs (train_simple / fine_tune / transfer) run end to end on CPU/gloo (dry-run slices)."""
import os

from mift.utils import harness


def _simple(rank, world, out):
    from mift.apps.labs import train_simple
    return train_simple(["--dry_run", "--model", "roberta-tiny", "--output_dir", out, "--max_steps", "3"])


def _fine(rank, world, out):
    from mift.apps.labs import fine_tune
    return fine_tune(["--dry_run", "--model", "gpt2-tiny", "--output_dir", out, "--max_steps", "2"])


def _transfer(rank, world, out):
    from mift.apps.labs import transfer
    return transfer(["--dry_run", "--base_model", "distilbert-tiny", "--output_dir", out])


def test_train_simple_ddp(tmp_path, monkeypatch):
    out = str(tmp_path / "m")
    r = harness.run(_simple, 2, out=out, env={"MIFT_AGNEWS": "synthetic"})
    assert len(r[0]) == 3 and os.path.exists(os.path.join(out, "model.safetensors"))


def test_fine_tune_full_params(tmp_path):
    out = str(tmp_path / "g")
    r = harness.run(_fine, 1, out=out)
    assert len(r[0]) >= 1 and os.path.exists(os.path.join(out, "config.json"))


def test_transfer_eval_each_epoch(tmp_path):
    out = str(tmp_path / "t")
    r = harness.run(_transfer, 2, out=out)
    assert len(r[0]["eval_accuracy"]) == 1 and os.path.exists(os.path.join(out, "model.safetensors"))
