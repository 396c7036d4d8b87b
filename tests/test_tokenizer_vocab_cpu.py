"""The WordPiece tokenizer built from a vocab.txt-format file keeps the whole vocabulary.

transformers 5 ignores ``BertTokenizerFast(vocab_file=...)`` and silently builds a 5-token vocabulary
(special tokens only), so every word became [UNK] and the tiny-BERT lab trained on constant inputs
(round 3: chance accuracy on the real AG-News arrow).  ``bert_tokenizer_from_vocab`` passes the
vocabulary as a dict and checks the size."""
import pytest

from mift.data.agnews import bert_tokenizer_from_vocab

pytest.importorskip("transformers")

WORDS = ["[PAD]", "[unused0]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", "stocks", "fell", "hello", "world", ",", "!",
         "##s", "stock"]


def test_vocab_file_is_loaded_whole(tmp_path):
    p = tmp_path / "vocab.txt"  # the HF cache stores it as an extension-less blob; the name does not matter
    p.write_text("\n".join(WORDS) + "\n", encoding="utf-8")
    tok = bert_tokenizer_from_vocab(str(p))
    assert tok.vocab_size == len(WORDS)
    ids = tok(["Hello world, stocks fell!"], max_length=16, padding="max_length", truncation=True)["input_ids"][0]
    assert ids[:8] == [3, 8, 9, 10, 6, 7, 11, 4]  # [CLS] hello world , stocks fell ! [SEP]
    assert 2 not in ids  # no [UNK]
