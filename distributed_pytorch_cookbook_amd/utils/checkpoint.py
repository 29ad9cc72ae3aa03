"""Checkpoint layout and resume.

Reference layout (``/root/reference/main-single.py:147-151``, same in every recipe): a flat
``torch.save(model.state_dict())`` at ``./checkpoints/checkpoint-%Y-%m-%d_%H-%M-%S.pt``
written by rank 0 at the end of training.  Every recipe here writes the same file with the
canonical *bare* keys (``embeddings.input_embeddings.weight``, ``decoder.layers.{i}.*``,
``norm_out.*``, ``lm_head.weight`` -- what the reference's FSDP path produced), whatever
the parallelism.  ``load_model_state`` also reads reference files, stripping the
``_orig_mod.`` (torch.compile) and ``module.`` (DDP) prefixes they carry.

Resume (absent in the reference): ``checkpoint-<ts>.train.pt`` next to the
model file holds optimizer moments (canonical flat layout), step / epoch counters and RNG
state, so an elastic restart continues instead of starting over.
"""
from __future__ import annotations

import glob
import os
from datetime import datetime
from pathlib import Path

import torch

PREFIXES = ("_orig_mod.", "module.")


def canonical_key(k: str) -> str:
    changed = True
    while changed:
        changed = False
        for p in PREFIXES:
            if k.startswith(p):
                k = k[len(p):]
                changed = True
    return k


def checkpoint_path(directory: str = "checkpoints", stamp: str | None = None, step: int | None = None) -> Path:
    """``checkpoint-<%Y-%m-%d_%H-%M-%S>[_step<N>].pt`` -- the reference's name, plus the
    optimizer step for periodic saves; an existing file is never overwritten (a ``.<n>``
    suffix is added instead)."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    stamp = stamp or datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    if step is not None:
        stamp = f"{stamp}_step{step}"
    path = d / f"checkpoint-{stamp}.pt"
    n = 1
    while path.exists():
        path = d / f"checkpoint-{stamp}.{n}.pt"
        n += 1
    return path


def save_model_state(state: dict, directory: str = "checkpoints", stamp: str | None = None,
                     step: int | None = None) -> Path:
    path = checkpoint_path(directory, stamp, step)
    cpu = {canonical_key(k): v.detach().to("cpu", copy=True).contiguous() for k, v in state.items()}
    tmp = path.with_suffix(".pt.tmp")
    torch.save(cpu, tmp)
    os.replace(tmp, path)
    return path


def load_model_state(path) -> dict:
    sd = torch.load(path, map_location="cpu", weights_only=True)
    return {canonical_key(k): v for k, v in sd.items()}


def train_state_path(model_path) -> Path:
    p = Path(model_path)
    return p.with_name(p.stem + ".train.pt")


def save_train_state(model_path, state: dict) -> Path:
    p = train_state_path(model_path)
    tmp = p.with_suffix(".tmp")
    torch.save(state, tmp)
    os.replace(tmp, p)
    return p


def load_train_state(model_path) -> dict | None:
    p = train_state_path(model_path)
    if not p.exists():
        return None
    return torch.load(p, map_location="cpu", weights_only=True)


def latest_checkpoint(directory: str = "checkpoints") -> Path | None:
    files = [f for f in glob.glob(os.path.join(directory, "checkpoint-*.pt")) if not f.endswith(".train.pt")]
    if not files:
        return None
    return Path(max(files, key=lambda f: (os.stat(f).st_mtime_ns, f)))


def rng_state() -> dict:
    st = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st: dict) -> None:
    torch.set_rng_state(st["cpu"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])
