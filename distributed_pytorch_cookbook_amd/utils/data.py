"""Datasets and tokenizer loading (reference ``/root/reference/data.py``).

``get_dataset`` / ``get_tokenizer`` / ``transform_dataset`` keep the reference
signatures and use Hugging Face ``datasets`` / ``transformers`` when the data is
available offline.  Otherwise -- and always with ``synthetic=True`` -- they produce a
deterministic synthetic token corpus of the same shape (rows of ``input_ids`` +
``attention_mask``), which is what every benchmark here uses (no network on the GPU box).

The synthetic sequences are drawn from a sparse first-order Markov chain over the full
GPT-2 vocabulary (each token has a few likely successors), so the LM has real structure
to learn and the training loss visibly falls, unlike uniform noise.
"""
from __future__ import annotations

from typing import Optional, Union

import torch
from torch.utils.data import Dataset

from .tokenizer import GPT2_VOCAB, ByteTokenizer


def _native_markov(i, seq_len, vocab, seed, branching):
    """Row i of the Markov corpus from the C++ runtime (None if it is unavailable)."""
    try:
        from ..runtime import synth_markov

        return synth_markov(1, seq_len, vocab, seed, branching, row0=int(i))[0]
    except Exception:
        return None


class SyntheticTokenDataset(Dataset):
    """``n`` rows of ``seq_len`` tokens; row i is a pure function of (seed, i)."""

    def __init__(self, n: int, seq_len: int, vocab_size: int = GPT2_VOCAB, seed: int = 0,
                 pad_fraction: float = 0.0, pad_id: int = 2, branching: int = 4):
        self.n, self.seq_len, self.vocab = n, seq_len, vocab_size
        self.seed, self.pad_fraction, self.pad_id = seed, pad_fraction, pad_id
        g = torch.Generator().manual_seed(1234567)
        # successor table: token t -> `branching` candidate next tokens
        self.succ = torch.randint(0, vocab_size, (vocab_size, branching), generator=g)
        self.branching = branching

    def __len__(self):
        return self.n

    def _succ_list(self):
        if getattr(self, "_succ_cache", None) is None:
            self._succ_cache = self.succ.tolist()
        return self._succ_cache

    def __getitem__(self, i):
        if self.pad_fraction == 0 and self.vocab > 0:
            ids = _native_markov(i, self.seq_len, self.vocab, self.seed, self.branching)
            if ids is not None:
                return {"input_ids": ids, "attention_mask": torch.ones(self.seq_len, dtype=torch.long)}
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + int(i))
        S = self.seq_len
        choice = torch.randint(0, self.branching, (S,), generator=g).tolist()
        noise = (torch.rand(S, generator=g) < 0.1).tolist()
        rnd = torch.randint(0, self.vocab, (S,), generator=g).tolist()
        succ = self._succ_list()
        out = [0] * S
        t = rnd[0]
        for s in range(S):
            out[s] = t
            t = rnd[s] if noise[s] else succ[t][choice[s]]
        ids = torch.tensor(out, dtype=torch.long)
        mask = torch.ones(S, dtype=torch.long)
        if self.pad_fraction > 0:
            L = int(S * (1.0 - self.pad_fraction * float(torch.rand((), generator=g))))
            L = max(L, 2)
            ids[L:] = self.pad_id
            mask[L:] = 0
        return {"input_ids": ids, "attention_mask": mask}


class FastSyntheticDataset(Dataset):
    """Same interface, vectorised generation (used by benchmarks with huge corpora)."""

    def __init__(self, n: int, seq_len: int, vocab_size: int = GPT2_VOCAB, seed: int = 0):
        self.n, self.seq_len, self.vocab, self.seed = n, seq_len, vocab_size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + int(i))
        ids = torch.randint(0, self.vocab, (self.seq_len,), generator=g)
        return {"input_ids": ids, "attention_mask": torch.ones(self.seq_len, dtype=torch.long)}


def get_tokenizer(name: str = "roneneldan/TinyStories-1M", max_length: int = 512, offline_stub: Optional[bool] = None):
    if not offline_stub:
        try:
            from transformers import GPT2Tokenizer

            tok = GPT2Tokenizer.from_pretrained(name, model_max_length=max_length, local_files_only=True)
            if tok.vocab_size < 256:  # an empty stand-in (no vocab files cached)
                raise OSError("tokenizer files not available offline")
            return tok
        except Exception:
            if offline_stub is False:
                raise
    return ByteTokenizer(model_max_length=max_length)


def get_dataset(name: str = "roneneldan/TinyStories", slice_size: Optional[Union[str, int]] = None,
                synthetic: Optional[bool] = None, seq_len: int = 256, n_train: int = 20000,
                n_val: int = 512, seed: int = 0, pad_fraction: float = 0.0):
    """(train, validation).  HF dataset if available offline (and not ``synthetic``)."""
    if not synthetic:
        try:
            import datasets

            split = f"train[:{slice_size}]" if slice_size is not None else "train"
            tr = datasets.load_dataset(name, split=split, download_mode="reuse_cache_if_exists")
            va = datasets.load_dataset(name, split="validation", download_mode="reuse_cache_if_exists")
            return tr, va
        except Exception:
            if synthetic is False:
                raise
    n = n_train
    if isinstance(slice_size, str) and slice_size.endswith("%"):
        n = max(1, int(n_train * float(slice_size[:-1]) / 100.0))
    elif isinstance(slice_size, int) or (isinstance(slice_size, str) and slice_size.isdigit()):
        n = int(slice_size)
    return (SyntheticTokenDataset(n, seq_len, seed=seed, pad_fraction=pad_fraction),
            SyntheticTokenDataset(n_val, seq_len, seed=seed + 99991, pad_fraction=pad_fraction))


def transform_dataset(dataset, tokenizer, max_length: int = 512, num_proc: int = 8):
    """Tokenise + pad to ``max_length`` (HF path); synthetic datasets pass through."""
    if isinstance(dataset, (SyntheticTokenDataset, FastSyntheticDataset)):
        return dataset

    def _tokenize(example):
        return tokenizer(example["text"], padding="max_length", max_length=max_length, truncation=True)

    dataset = dataset.map(_tokenize, batched=True, remove_columns=["text"], num_proc=num_proc)
    dataset.set_format("pt")
    return dataset
