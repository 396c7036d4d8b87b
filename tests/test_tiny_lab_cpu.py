"""Tiny-BERT lab on CPU/gloo: HF parity of the model, 2-rank DDP train -> save -> 2-rank DDP infer."""
import os

import pytest
import torch

from mift.models.bert import BertConfig, BertForSequenceClassification
from mift.obs.tb import read_events
from mift.utils import harness


def test_bert_matches_hf():
    transformers = pytest.importorskip("transformers")
    c = BertConfig.tiny(vocab_size=500)
    m = BertForSequenceClassification(c).init_weights(0).eval()
    hc = transformers.BertConfig(vocab_size=500, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                 intermediate_size=256, max_position_embeddings=256, num_labels=4)
    hf = transformers.BertForSequenceClassification(hc).eval()
    missing, unexpected = hf.load_state_dict(m.state_dict(), strict=False)
    assert not [k for k in missing if "position_ids" not in k], missing
    ids = torch.randint(0, 500, (3, 20))
    am = torch.ones_like(ids)
    am[1, 12:] = 0
    with torch.no_grad():
        torch.testing.assert_close(m(input_ids=ids, attention_mask=am)["logits"],
                                   hf(input_ids=ids, attention_mask=am).logits, atol=1e-5, rtol=1e-4)


def _train(rank, world, out):
    from mift.apps.tiny_lab import train
    return train(["--epochs", "2", "--subset", "256", "--batch", "16", "--out", out, "--eval_rows", "128"])


def _infer(rank, world, out):
    from mift.apps.tiny_lab import infer
    return infer(["--ckpt", out, "--max_test", "200", "--batch", "32"])


def test_tiny_lab_ddp_roundtrip(tmp_path, capfd):
    out = str(tmp_path / "tiny_out")
    r = harness.run(_train, 2, out=out)
    assert os.path.exists(os.path.join(out, "model.safetensors")) and os.path.exists(os.path.join(out, "config.json"))
    assert os.path.exists(os.path.join(out, "log.rank1.txt"))
    ev = [f for f in os.listdir(os.path.join(out, "tb", "rank0"))]
    recs = read_events(os.path.join(out, "tb", "rank0", ev[0]))
    assert any("loss" in s for _, s in recs) and any("eval_accuracy" in s for _, s in recs)
    assert r[0]["accuracy"] == r[1]["accuracy"]
    i = harness.run(_infer, 2, out=out)
    assert i[0]["samples"] == 200
    text = capfd.readouterr().out
    assert "[RANK 0] TRAIN_RUNTIME_SEC=" in text and "[RANK 0] EVAL accuracy=" in text
    assert "[RANK 0] INFER global_accuracy=" in text and "step_ms=" in text and "[RANK 1] WORLD_SIZE=2" in text
