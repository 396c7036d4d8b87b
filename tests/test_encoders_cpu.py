"""RoBERTa / DistilBERT classifier parity vs transformers (logits + loss, padded batch)."""
import pytest
import torch

from mift.models.encoders import (DistilBertConfig, DistilBertForSequenceClassification, RobertaConfig,
                                  RobertaForSequenceClassification)


def _batch(vocab, pad):
    ids = torch.randint(3, vocab, (3, 17))
    am = torch.ones_like(ids)
    am[1, 12:] = 0
    ids[1, 12:] = pad
    return ids, am, torch.tensor([0, 3, 1])


def _cmp(m, hf, pad):
    ids, am, lab = _batch(m.config.vocab_size, pad)
    with torch.no_grad():
        o = m(input_ids=ids, attention_mask=am, labels=lab)
        r = hf(input_ids=ids, attention_mask=am, labels=lab)
    torch.testing.assert_close(o["logits"], r.logits, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(o["loss"], r.loss, atol=1e-5, rtol=1e-5)


def test_roberta_matches_hf():
    transformers = pytest.importorskip("transformers")
    c = RobertaConfig.preset("roberta-tiny", num_labels=4)
    m = RobertaForSequenceClassification(c).init_weights(0).eval()
    hc = transformers.RobertaConfig(vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                                    num_hidden_layers=c.num_hidden_layers, num_attention_heads=c.num_attention_heads,
                                    intermediate_size=c.intermediate_size,
                                    max_position_embeddings=c.max_position_embeddings, type_vocab_size=1,
                                    num_labels=4, pad_token_id=1, layer_norm_eps=1e-5)
    hf = transformers.RobertaForSequenceClassification(hc).eval()
    missing, _ = hf.load_state_dict(m.state_dict(), strict=False)
    assert not [k for k in missing if "position_ids" not in k], missing
    _cmp(m, hf, 1)


def test_distilbert_matches_hf():
    transformers = pytest.importorskip("transformers")
    c = DistilBertConfig.preset("distilbert-tiny", num_labels=4)
    m = DistilBertForSequenceClassification(c).init_weights(0).eval()
    hc = transformers.DistilBertConfig(vocab_size=c.vocab_size, dim=c.dim, n_layers=c.n_layers, n_heads=c.n_heads,
                                       hidden_dim=c.hidden_dim, max_position_embeddings=c.max_position_embeddings,
                                       num_labels=4)
    hf = transformers.DistilBertForSequenceClassification(hc).eval()
    missing, _ = hf.load_state_dict(m.state_dict(), strict=False)
    assert not [k for k in missing if "position_ids" not in k], missing
    _cmp(m, hf, 0)
