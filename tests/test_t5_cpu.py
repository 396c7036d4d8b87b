"""T5/FLAN-T5 parity vs transformers (logits, loss, greedy generate) on a tiny random config."""
import pytest
import torch

from mift.models.t5 import T5Config, T5ForConditionalGeneration


def _pair():
    transformers = pytest.importorskip("transformers")
    c = T5Config.preset("t5-tiny")
    m = T5ForConditionalGeneration(c).init_weights(0).eval()
    hc = transformers.T5Config(vocab_size=c.vocab_size, d_model=c.d_model, d_kv=c.d_kv, d_ff=c.d_ff,
                               num_layers=c.num_layers, num_decoder_layers=c.num_decoder_layers,
                               num_heads=c.num_heads, feed_forward_proj="gated-gelu", tie_word_embeddings=False,
                               dropout_rate=0.0, decoder_start_token_id=0, pad_token_id=0, eos_token_id=1)
    hc.tie_word_embeddings = False  # FLAN-T5: untied head (kwarg not honoured by every transformers version)
    hf = transformers.T5ForConditionalGeneration(hc).eval()
    assert hf.lm_head.weight.data_ptr() != hf.shared.weight.data_ptr()
    sd = m.state_dict()
    missing, _ = hf.load_state_dict(sd, strict=False)
    assert not [k for k in missing if "embed_tokens" not in k], missing
    hf.encoder.embed_tokens = hf.shared  # HF ties these; be explicit across versions
    hf.decoder.embed_tokens = hf.shared
    return m, hf


def test_t5_logits_and_loss_match_hf():
    m, hf = _pair()
    ids = torch.randint(2, 512, (2, 11))
    am = torch.ones_like(ids)
    am[1, 8:] = 0
    lab = torch.randint(2, 512, (2, 6))
    lab[0, 4:] = -100
    with torch.no_grad():
        o = m(input_ids=ids, attention_mask=am, labels=lab)
        r = hf(input_ids=ids, attention_mask=am, labels=lab)
    torch.testing.assert_close(o["logits"], r.logits, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(o["loss"], r.loss, atol=1e-5, rtol=1e-5)


def test_t5_generate_matches_hf():
    m, hf = _pair()
    ids = torch.randint(2, 512, (3, 9))
    am = torch.ones_like(ids)
    ours = m.generate(ids, am, max_new_tokens=12, eos_token_id=-1)
    theirs = hf.generate(input_ids=ids, attention_mask=am, max_new_tokens=12, do_sample=False, eos_token_id=None)
    assert torch.equal(ours, theirs)
