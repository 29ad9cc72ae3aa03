"""Offline GPT-2-sized tokenizer stub.

The reference loads ``GPT2Tokenizer.from_pretrained("roneneldan/TinyStories-1M")``
(``/root/reference/data.py:18-20``), which needs the Hugging Face hub.  Without network
(or an HF cache) we fall back to this byte-level tokenizer with the same interface the
recipes use: ``vocab_size`` 50257, ``eos_token_id`` 50256, settable ``pad_token_id``,
``__call__(texts, truncation, max_length, padding, return_tensors)`` returning
``input_ids`` / ``attention_mask`` and ``decode(ids, skip_special_tokens)``.
"""
from __future__ import annotations

import torch

GPT2_VOCAB = 50257
GPT2_EOS = 50256
BYTE_OFFSET = 256  # ids 0..255 stay free (the reference uses pad id 2)


class ByteTokenizer:
    def __init__(self, model_max_length: int = 512, vocab_size: int = GPT2_VOCAB):
        self.vocab_size = vocab_size
        self.eos_token_id = vocab_size - 1
        self.pad_token_id = self.eos_token_id
        self.model_max_length = model_max_length
        self.name_or_path = "byte-level-offline-stub"

    def encode(self, text: str) -> list[int]:
        return [BYTE_OFFSET + b for b in text.encode("utf-8")]

    def __call__(self, texts, truncation=False, max_length=None, padding=False, return_tensors=None):
        single = isinstance(texts, str)
        texts = [texts] if single else list(texts)
        max_length = max_length or self.model_max_length
        ids = [self.encode(t) for t in texts]
        if truncation:
            ids = [x[:max_length] for x in ids]
        if padding == "max_length":
            tgt = max_length
        elif padding is True or padding == "longest":
            tgt = max(len(x) for x in ids)
        else:
            tgt = None
        masks = [[1] * len(x) for x in ids]
        if tgt is not None:
            masks = [m + [0] * (tgt - len(m)) for m in masks]
            ids = [x + [self.pad_token_id] * (tgt - len(x)) for x in ids]
        out = {"input_ids": ids, "attention_mask": masks}
        if return_tensors == "pt":
            out = {k: torch.tensor(v, dtype=torch.long) for k, v in out.items()}
        elif single:
            out = {k: v[0] for k, v in out.items()}
        return out

    def decode(self, ids, skip_special_tokens=False) -> str:
        if torch.is_tensor(ids):
            ids = ids.tolist()
        bs = bytearray()
        for i in ids:
            if BYTE_OFFSET <= i < BYTE_OFFSET + 256:
                bs.append(i - BYTE_OFFSET)
            elif not skip_special_tokens:
                bs.extend(f"<{i}>".encode())
        return bs.decode("utf-8", errors="replace")
