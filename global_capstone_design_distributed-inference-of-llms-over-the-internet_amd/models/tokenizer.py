"""Tokenizer resolution without network access.

The reference calls ``AutoTokenizer.from_pretrained(args.model)`` (src/main.py:98-100).
Here a local HF directory's tokenizer is used when present (``local_files_only``); for
presets / synthetic weights a byte-level tokenizer (UTF-8 bytes + 3 specials) stands in,
which is exact and reversible for any text.
"""
from __future__ import annotations

import logging
import os
from typing import List

logger = logging.getLogger(__name__)


class ByteTokenizer:
    PAD, BOS, EOS, OFFSET = 0, 1, 2, 3

    def __init__(self, vocab_size: int, eos_token_id: int = 2, bos_token_id: int = 1):
        self.vocab_size = vocab_size
        self.eos_token_id = eos_token_id if eos_token_id < vocab_size else self.EOS
        self.bos_token_id = bos_token_id if bos_token_id < vocab_size else self.BOS
        self.pad_token_id = self.PAD

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = [b + self.OFFSET for b in text.encode("utf-8")]
        ids = [i % self.vocab_size for i in ids]
        return ([self.bos_token_id] if add_bos else []) + ids

    def __call__(self, text: str, return_tensors=None):
        import torch

        ids = self.encode(text)

        class _Enc:
            pass

        enc = _Enc()
        enc.input_ids = torch.tensor([ids]) if return_tensors == "pt" else [ids]
        return enc

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        out = bytearray()
        for i in ids:
            i = int(i)
            if self.OFFSET <= i < self.OFFSET + 256:
                out.append(i - self.OFFSET)
            elif not skip_special_tokens or i >= self.OFFSET + 256:
                out.extend(f"<{i}>".encode())
        return out.decode("utf-8", errors="replace")


def load_tokenizer(model: str, cfg=None):
    if os.path.isdir(model):
        try:
            from transformers import AutoTokenizer

            tok = AutoTokenizer.from_pretrained(model, local_files_only=True)
            if tok.pad_token is None:
                tok.pad_token = tok.eos_token
            return tok
        except Exception as e:
            logger.warning(f"no usable tokenizer in {model} ({e}); using byte-level tokenizer")
    vocab = cfg.vocab_size if cfg is not None else 32000
    eos = cfg.eos_token_id if cfg is not None else 2
    bos = cfg.bos_token_id if cfg is not None else 1
    return ByteTokenizer(vocab, eos, bos)
