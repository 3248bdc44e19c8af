"""`ASRBPEMixin._setup_tokenizer` (reference nemo/collections/asr/parts/mixins/mixins.py:49-140) for
the BPE model shells: `tokenizer.type: bpe` loads `<dir>/tokenizer.model` with SentencePiece (the
reference's SentencePieceTokenizer); `wpe` reads `<dir>/vocab.txt` (WordPiece: `##` continues a
word).  Aggregate (multilingual) tokenizers and HF kwargs are out of scope (tokenizers).
"""
from __future__ import annotations

import os
from typing import Dict, List


class SentencePieceTokenizer:
    """nemo/collections/common/tokenizers/sentencepiece_tokenizer.py (the id <-> text subset)."""

    def __init__(self, model_path: str):
        import sentencepiece as spm
        if not os.path.exists(model_path):
            raise FileNotFoundError(f"tokenizer model {model_path} not found")
        self.tokenizer = spm.SentencePieceProcessor()
        self.tokenizer.Load(model_path)
        self.vocab_size = self.tokenizer.get_piece_size()

    def get_vocab(self) -> Dict[str, int]:
        return {self.tokenizer.id_to_piece(i): i for i in range(self.vocab_size)}

    def text_to_ids(self, text: str) -> List[int]:
        return list(self.tokenizer.encode_as_ids(text))

    def ids_to_text(self, ids: List[int]) -> str:
        return self.tokenizer.decode_ids([int(i) for i in ids])


class WordPieceTokenizer:
    """A vocab.txt WordPiece vocabulary (one token per line; `##x` continues the previous word)."""

    def __init__(self, vocab_path: str):
        with open(vocab_path, encoding="utf-8") as f:
            self.vocab = [ln.rstrip("\n") for ln in f if ln.strip()]
        self._ids = {t: i for i, t in enumerate(self.vocab)}
        self.vocab_size = len(self.vocab)

    def get_vocab(self) -> Dict[str, int]:
        return dict(self._ids)

    def ids_to_text(self, ids: List[int]) -> str:
        out = ""
        for i in ids:
            t = self.vocab[int(i)]
            out += t[2:] if t.startswith("##") else ((" " if out else "") + t)
        return out


class ASRBPEMixin:
    def _setup_tokenizer(self, tokenizer_cfg) -> None:
        ttype = tokenizer_cfg.get("type")
        if ttype is None:
            raise ValueError("`tokenizer.type` cannot be None")
        ttype = str(ttype).lower()
        if ttype not in ("bpe", "wpe"):
            raise ValueError("`tokenizer.type` must be either `bpe` for SentencePiece tokenizer or `wpe` for BERT "
                             "based tokenizer")
        tdir = tokenizer_cfg["dir"]        # `???` in the yamls: MissingMandatoryValue until set
        self.tokenizer_dir, self.tokenizer_type = tdir, ttype
        # the files are registered as .nemo artifacts (mixins.py:85-151): save_to packs them, a restored
        # config's `nemo:` paths resolve to the archive's copies (no dependency on the original dir)
        if ttype == "bpe":
            path = tokenizer_cfg.get("model_path") or os.path.join(tdir, "tokenizer.model")
            path = self.register_artifact("tokenizer.model_path", path)
            for key, default in (("vocab_path", "vocab.txt"), ("spe_tokenizer_vocab", "tokenizer.vocab")):
                self.register_artifact("tokenizer." + key, tokenizer_cfg.get(key) or os.path.join(tdir, default),
                                       verify_src_exists=False)
            self.tokenizer = SentencePieceTokenizer(path)
        else:
            path = tokenizer_cfg.get("vocab_path") or os.path.join(tdir, "vocab.txt")
            path = self.register_artifact("tokenizer.vocab_path", path)
            self.tokenizer = WordPieceTokenizer(path)

    def _tokenizer_vocabulary(self) -> List[str]:
        vocab = self.tokenizer.get_vocab()
        return [t for t, _ in sorted(vocab.items(), key=lambda kv: kv[1])]
