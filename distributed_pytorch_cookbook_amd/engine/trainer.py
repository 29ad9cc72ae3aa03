"""The shared train / eval / generate / checkpoint loop of every recipe.

Reference loop: ``/root/reference/main-single.py:80-151`` (and its copies in
``main-ddp.py:105-185``, ``main-fsdp.py:117-200``, ``main-pipe.py:150-221``):
tqdm per epoch with ``[training] Epoch e/E | loss: x.xxx`` refreshed every
``PRINT_FREQ = 8`` steps, validation loss / accuracy, three greedy samples, a final
rank-0 ``torch.save``.  Kept here, with: the PRINT_FREQ averaging off-by-one fixed,
a per-epoch reshuffle (the reference never called ``set_epoch``) whose global batches do
not depend on the world size (``GlobalBatchSampler``), metrics reduced in ONE collective per epoch
instead of two per batch, generation run on every rank when the engine needs it
(FSDP, pipeline) so no collective is left unmatched, tokens/s reported, and
``--resume`` / ``--max_steps`` support.
"""
from __future__ import annotations

import json
import math
import os
import time

import torch
from torch.utils.data import DataLoader, Sampler

from ..parallel.transport import check_peer_comms
from ..parallel import comm
from ..utils.batch import generate, prepare_batch
from ..utils.checkpoint import (latest_checkpoint, load_model_state, load_train_state, rng_state,
                                save_model_state, save_train_state, set_rng_state)
from ..utils.metrics import mfu, peak_memory_gib, train_flops_per_token
from ..utils.profiling import StepProfiler, mark, maybe_inject_fault

PRINT_FREQ = 8
PROMPTS = ("The big brown cat ", "One day, ", "She said ")


def _tqdm(it, enabled):
    if not enabled:
        return it
    try:
        from tqdm import tqdm

        return tqdm(it)
    except Exception:  # pragma: no cover
        return it


class _NoBar:
    def __init__(self, it):
        self.it = it

    def __iter__(self):
        return iter(self.it)

    def set_description(self, s):
        pass


class GlobalBatchSampler(Sampler):
    """Data-parallel sampler whose global batches do not depend on the world size.

    The reference shards with ``DistributedSampler`` (``/root/reference/main-ddp.py:83-84``),
    which deals a shuffled order round-robin, so W ranks x B sequences see different global
    batches than one process at W x B.  Here epoch e's order is ``randperm(n)`` of a generator
    seeded ``seed + e`` -- exactly the order a single-process ``DataLoader(shuffle=True)``
    with that generator produces -- and global batch i is its slice [i W B, (i + 1) W B), of
    which rank r takes the r-th B sequences.  A DDP / FSDP / PP x DP run therefore trains on
    the same global batches as ``main-single.py`` at batch W x B (the multi-rank recipe tests
    compare their checkpoints), and resume positions are global batch indices.  Incomplete
    global batches are dropped (``drop_last``)."""

    def __init__(self, n: int, batch_size: int, world: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 0):
        self.n, self.B, self.W, self.r = n, batch_size, max(1, world), rank
        self.shuffle, self.seed, self.epoch = shuffle, seed, 0
        self.nb = n // (self.B * self.W)

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g)
        else:
            order = torch.arange(self.n)
        gb = self.B * self.W
        for i in range(self.nb):
            yield from order[i * gb + self.r * self.B:i * gb + (self.r + 1) * self.B].tolist()

    def __len__(self):
        return self.nb * self.B


def make_loader(ds, batch_size, num_workers, dp_world, dp_rank, shuffle, seed, device):
    sampler = GlobalBatchSampler(len(ds), batch_size, dp_world, dp_rank, shuffle, seed)
    return DataLoader(ds, batch_size=batch_size, sampler=sampler, num_workers=num_workers,
                      pin_memory=device.type == "cuda", drop_last=True,
                      persistent_workers=num_workers > 0), sampler


class Trainer:
    def __init__(self, args, engine, tokenizer, pad_id: int = 2):
        self.args, self.engine, self.tok, self.pad_id = args, engine, tokenizer, pad_id
        self.device = engine.device
        self.log = engine.is_logger
        self.start_epoch = 0
        self.skip_batches = 0  # batches of start_epoch already trained (mid-epoch resume)
        self.history = []
        vocab = getattr(tokenizer, "vocab_size", 50257)
        self.flops_per_token = train_flops_per_token(args.dim, args.heads, args.head_dim, args.num_layers,
                                                     vocab, args.sequence_length)

    # ------------------------------------------------------------------ helpers
    def _jsonl(self, rec):
        if self.log and self.args.log_jsonl:
            with open(self.args.log_jsonl, "a") as f:
                f.write(json.dumps(rec) + "\n")

    def maybe_resume(self):
        if not self.args.resume:
            return
        path = latest_checkpoint(self.args.checkpoint_dir) if self.args.resume == "latest" else self.args.resume
        if path is None:
            if self.log:
                print("[resume] no checkpoint found; starting fresh")
            return
        self.engine.load_model_state(load_model_state(path))
        st = load_train_state(path)
        if st is not None:
            self.engine.load_train_state(st)
            self.start_epoch = int(st.get("epoch", 0))
            self.skip_batches = int(st.get("batch", 0))
            rng = st.get("rng_per_rank")
            if rng is not None and len(rng) == comm.world_size():
                set_rng_state(rng[comm.rank()])  # each rank its own stream
            elif "rng" in st and comm.world_size() == 1:
                set_rng_state(st["rng"])
        if self.log:
            print(f"[resume] loaded {path} (epoch {self.start_epoch}, batch {self.skip_batches})")

    # ------------------------------------------------------------------ main loop
    def fit(self, train_ds, val_ds):
        a = self.args
        e = self.engine
        self.maybe_resume()
        if getattr(a, "data_path", None):
            # pre-tokenised corpus through the native mmap loader (runtime/csrc/runtime.cpp)
            from itertools import islice

            from ..runtime import NativeBatchLoader, TokenFile

            tf = TokenFile(a.data_path, a.token_bytes)
            steps = a.max_steps or max(1, a.train_samples // (a.batch_size * e.dp_world))
            tl = NativeBatchLoader(tf, a.batch_size, a.sequence_length, a.seed, e.dp_rank, e.dp_world)
            vl = NativeBatchLoader(tf, a.batch_size, a.sequence_length, a.seed + 7919, e.dp_rank, e.dp_world)
            vsteps = a.eval_steps or max(1, a.val_samples // (a.batch_size * e.dp_world))

            class _Epoch:
                """Epoch e of the stream: batches [e * n, (e + 1) * n), positioned by seek, so
                a mid-epoch resume reads exactly the batches the uninterrupted run would."""

                def __init__(self, loader, n, per_epoch=True):
                    self.loader, self.n, self.per_epoch = loader, n, per_epoch
                    self.epoch, self.start = 0, 0

                def position(self, epoch, start=0):
                    self.epoch, self.start = epoch, start

                def __iter__(self):
                    self.loader.seek((self.epoch * self.n if self.per_epoch else 0) + self.start)
                    return islice(self.loader, self.n - self.start)

                def __len__(self):
                    return self.n - self.start

            train_loader, sampler = _Epoch(tl, steps), None
            val_loader = _Epoch(vl, vsteps, per_epoch=False)  # the same held-out batches each epoch
        else:
            train_loader, sampler = make_loader(train_ds, a.batch_size, a.num_workers, e.dp_world, e.dp_rank,
                                                True, a.seed, self.device)
            val_loader, _ = make_loader(val_ds, a.batch_size, min(a.num_workers, 2), e.dp_world, e.dp_rank,
                                        False, a.seed, self.device)
        for ei in range(self.start_epoch, a.epochs):
            if sampler is not None:
                # the shuffle order is a function of (seed, epoch) alone, so a resumed run sees
                # the same batches as an uninterrupted one
                sampler.set_epoch(ei)
            skip = self.skip_batches if ei == self.start_epoch else 0
            if hasattr(train_loader, "position"):  # native stream: seek past the trained batches
                train_loader.position(ei, skip)
                self.train_epoch(ei, train_loader, skip=skip, preskipped=True)
            else:
                self.train_epoch(ei, train_loader, skip=skip)
            self.validate(ei, val_loader)
            if not a.no_generate:
                self.sample()
            comm.barrier()
        comm.barrier()
        path = None
        if not a.no_save:
            path = self.save(a.epochs)
        return path

    def train_epoch(self, ei, loader, skip: int = 0, preskipped: bool = False):
        a, e = self.args, self.engine
        e.model.train()  # reference main-single.py:35 / main-ddp.py:109 (dropout on)
        pb = _tqdm(loader, self.log) if self.log else _NoBar(loader)
        pb.set_description(f"[training] Epoch {ei+1}/{a.epochs} | loss: ?????")
        window, nwin = None, 0
        t0 = time.perf_counter()
        tokens = 0
        prof = StepProfiler(a.profile if ei == self.start_epoch else None, comm.rank())
        for i, batch in enumerate(pb, start=skip if preskipped else 0):
            if a.max_steps and i >= a.max_steps:
                break
            if i < skip:  # trained before the checkpoint this run resumed from
                continue
            maybe_inject_fault(e.step_count, comm.rank())
            inputs, targets = prepare_batch(batch, self.pad_id, self.device)
            with mark("train_step"):
                loss = e.train_step(inputs, targets)
            prof.step()
            if getattr(a, "save_every", 0) and e.step_count % a.save_every == 0:
                self.save(ei, batch=i + 1)  # resume continues this epoch after batch i
            tokens += targets.numel() * e.dp_world
            if loss is not None:
                window = loss if window is None else window + loss
                nwin += 1
            if (i + 1) % PRINT_FREQ == 0:
                avg = self._window_loss(window, nwin)
                if self.device.type == "cuda":
                    torch.cuda.synchronize()
                    check_peer_comms()  # (a peer-access wait that gave up would leave wrong data)
                dt = time.perf_counter() - t0
                tps = tokens / dt if dt > 0 else 0.0
                util = mfu(tps / max(comm.world_size(), 1), self.flops_per_token)
                pb.set_description(f"[training] Epoch {ei+1}/{a.epochs} | loss: {avg:.3f} | tok/s: {tps:,.0f}"
                                   f" | MFU {100 * util:.1f}%")
                rec = {"epoch": ei + 1, "step": e.step_count, "loss": avg, "tokens_per_s": tps,
                       "tokens_per_s_per_gpu": tps / max(comm.world_size(), 1), "mfu": util,
                       "step_ms": 1000.0 * dt / PRINT_FREQ, "peak_mem_gib": peak_memory_gib(self.device)}
                self.history.append(rec)
                self._jsonl(rec)
                window, nwin, tokens, t0 = None, 0, 0, time.perf_counter()
        prof.close()
        if self._pipelined() or (window is not None and nwin):  # (a collective for pipelines: every rank)
            avg = self._window_loss(window, nwin)
            if avg == avg:
                self.history.append({"epoch": ei + 1, "step": e.step_count, "loss": avg})

    def _pipelined(self) -> bool:
        return getattr(self.engine, "pp", 1) > 1 and comm.world_size() > 1

    def _window_loss(self, window, nwin) -> float:
        """Mean training loss of the last window.  A pipeline's loss exists only on its last stage
        (one per replica) while rank 0 -- the logger -- holds the first: the window sums and counts
        are summed over the world (the other stages add zeros), one collective on every rank."""
        if not self._pipelined():
            return (window / max(nwin, 1)).item() if window is not None else float("nan")
        ws = window if window is not None else torch.zeros((), device=self.device)
        red = comm.all_reduce_scalars([ws, float(nwin if window is not None else 0)], self.device)
        n = float(red[1])
        return float(red[0]) / n if n > 0 else float("nan")

    @torch.no_grad()
    def validate(self, ei, loader):
        a, e = self.args, self.engine
        e.model.eval()  # reference main-ddp.py:135 (dropout off for validation and sampling)
        tot = torch.zeros(3, device=self.device)
        pb = _tqdm(loader, self.log) if self.log else _NoBar(loader)
        pb.set_description(f"[validation] Epoch {ei+1}/{a.epochs} | loss: ?????, accuracy: ?????")
        for i, batch in enumerate(pb):
            if a.eval_steps and i >= a.eval_steps:
                break
            inputs, targets = prepare_batch(batch, self.pad_id, self.device)
            r = e.eval_step(inputs, targets)
            if r is not None:
                tot += torch.stack([x.float().reshape(()) for x in r])
        red = comm.all_reduce_scalars(list(tot), self.device, group=None)
        # every stage holds zeros except the loss-holding ranks, so a global sum is exact
        loss_sum, n, correct = (float(x) for x in red.tolist())
        loss = loss_sum / max(n, 1.0)
        acc = 100.0 * correct / max(n, 1.0)
        if self.log:
            msg = f"[validation] Epoch {ei+1}/{a.epochs} | loss: {loss:.3f}, accuracy: {acc:.2f}"
            pb.set_description(msg)
            print(msg)
        rec = {"epoch": ei + 1, "val_loss": loss, "val_accuracy": acc}
        self.history.append(rec)
        self._jsonl(rec)
        return loss, acc

    def sample(self):
        e = self.engine
        if not (e.collective_generate or self.log):
            return
        if self.log:
            print("Argmax sampling from model")
        for p in PROMPTS:
            s = generate(e.lm(), p, self.tok, self.device)
            if self.log:
                print(s)

    def save(self, epoch, batch: int = 0):
        sd = self.engine.full_state_dict()
        path = None
        tstate = self.engine.train_state()
        rngs = comm.gather_objects(rng_state())  # every rank's RNG streams (collective)
        if self.log and sd is not None:
            # periodic saves carry the step in the name: two within one second never collide
            path = save_model_state(sd, self.args.checkpoint_dir, step=self.engine.step_count if batch else None)
            tstate = dict(tstate or {})
            tstate.update({"epoch": epoch, "batch": batch, "rng": rng_state(), "rng_per_rank": rngs})
            save_train_state(path, tstate)
            print(f"saved {path}")
        comm.barrier()
        return path
