"""Tokenizer loading (offline-safe).

Resolution order for ``load_tokenizer(name_or_path)``:
  1. a directory with ``tokenizer.json`` (ours or HF fast tokenizer);
  2. ``transformers.AutoTokenizer.from_pretrained(..., local_files_only=True)``
     (an HF cache that already holds the reference tokenizer);
  3. a byte-level BPE (GPT-2 style) trained on the corpus itself with the
     ``tokenizers`` library — no network; ids stay < the model vocab.
Pad = EOS as in the reference (``tok.pad_token = tok.eos_token``).
"""
import json
import os


class Tok:
    def __init__(self, tk, eos_token="<|endoftext|>", name="bpe"):
        self.tk = tk
        self.eos_token = eos_token
        self.eos_id = tk.token_to_id(eos_token)
        if self.eos_id is None:
            self.eos_id = 0
        self.pad_id = self.eos_id
        self.name = name

    @property
    def vocab_size(self):
        return self.tk.get_vocab_size()

    def encode(self, text):
        return self.tk.encode(text).ids

    def encode_batch(self, texts):
        return [e.ids for e in self.tk.encode_batch(list(texts))]

    def decode(self, ids):
        return self.tk.decode(list(ids))

    def save_pretrained(self, d):
        os.makedirs(d, exist_ok=True)
        self.tk.save(os.path.join(d, "tokenizer.json"))
        with open(os.path.join(d, "tokenizer_config.json"), "w") as f:
            json.dump({"tokenizer_class": "PreTrainedTokenizerFast", "eos_token": self.eos_token,
                       "pad_token": self.eos_token, "bos_token": self.eos_token, "padding_side": "right",
                       "model_max_length": 1024}, f, indent=2)
        with open(os.path.join(d, "special_tokens_map.json"), "w") as f:
            json.dump({"eos_token": self.eos_token, "pad_token": self.eos_token, "bos_token": self.eos_token}, f)


class HFTok(Tok):
    def __init__(self, hf):
        self.hf = hf
        if hf.pad_token is None:
            hf.pad_token = hf.eos_token
        hf.padding_side = "right"
        self.eos_token = hf.eos_token
        self.eos_id = hf.eos_token_id
        self.pad_id = hf.pad_token_id
        self.name = getattr(hf, "name_or_path", "hf")

    @property
    def vocab_size(self):
        return len(self.hf)

    def encode(self, text):
        return self.hf(text)["input_ids"]

    def encode_batch(self, texts):
        return self.hf(list(texts))["input_ids"]

    def decode(self, ids):
        return self.hf.decode(list(ids))

    def save_pretrained(self, d):
        self.hf.save_pretrained(d)


def train_bpe(lines, vocab_size=50257, min_frequency=2):
    from tokenizers import ByteLevelBPETokenizer
    tk = ByteLevelBPETokenizer()
    tk.train_from_iterator((ln for ln in lines if ln), vocab_size=vocab_size, min_frequency=min_frequency,
                           special_tokens=["<|endoftext|>"], show_progress=False)
    return Tok(tk._tokenizer if hasattr(tk, "_tokenizer") else tk, name="bpe-trained")


def load_tokenizer(name_or_path, corpus_lines=None, vocab_size=50257):
    if name_or_path and os.path.isdir(name_or_path) and os.path.exists(os.path.join(name_or_path, "tokenizer.json")):
        from tokenizers import Tokenizer
        tk = Tokenizer.from_file(os.path.join(name_or_path, "tokenizer.json"))
        eos = "<|endoftext|>"
        cfgp = os.path.join(name_or_path, "tokenizer_config.json")
        if os.path.exists(cfgp):
            with open(cfgp) as f:
                e = json.load(f).get("eos_token")
                if isinstance(e, dict):
                    e = e.get("content")
                eos = e or eos
        return Tok(tk, eos, name=name_or_path)
    try:
        from transformers import AutoTokenizer
        hf = AutoTokenizer.from_pretrained(name_or_path, local_files_only=True, use_fast=True)
        return HFTok(hf)
    except Exception:
        pass
    if corpus_lines is None:
        corpus_lines = ["hello world"]
    return train_bpe(corpus_lines, vocab_size=vocab_size)
