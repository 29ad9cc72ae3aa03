"""Command-line flags shared by the five recipes.

The first block is the reference's flag set with identical names and defaults
(``/root/reference/main-single.py:154-170``; ``--cpu_offload`` from ``main-fsdp.py:219``).
The second block is new: model presets, synthetic data, step limits, seeding, resume,
parallelism shape and tuning knobs.
"""
from __future__ import annotations

import argparse
import os

from .models.gpt import PRESETS


def build_parser(recipe: str = "single") -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=f"MI355X cookbook recipe: {recipe}")
    # --- reference flags (same names, same defaults)
    p.add_argument("--batch_size", type=int, default=64)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--sequence_length", type=int, default=256)
    p.add_argument("--dim", type=int, default=256)
    p.add_argument("--head_dim", type=int, default=32)
    p.add_argument("--heads", type=int, default=8)
    p.add_argument("--num_layers", type=int, default=8)
    p.add_argument("--learning_rate", type=float, default=1e-4)
    p.add_argument("--dataset_slice", type=str, default="100%")
    p.add_argument("--num_workers", type=int, default=4)
    p.add_argument("--disable_amp", action="store_true",
                   help="f32 compute: the f32-input MFMA GEMM and f32 flash-attention kernels "
                        "instead of the bf16 ones")
    p.add_argument("--disable_compile", action="store_true",
                   help="do not capture the train step into a HIP graph")
    if recipe == "fsdp":
        p.add_argument("--cpu_offload", action="store_true",
                       help="keep f32 master shards + optimizer state in pinned host memory")
    # --- new flags
    p.add_argument("--model", type=str, default=None, choices=sorted(PRESETS),
                   help="architecture preset (overrides dim/head_dim/heads/num_layers/sequence_length)")
    p.add_argument("--activation", type=str, default=None, choices=["relu", "gelu"])
    p.add_argument("--graph", action="store_true",
                   help="(kept for old command lines: the step is captured into a HIP graph on every "
                        "rank by default, RCCL collectives inside; --disable_compile runs eager steps)")
    p.add_argument("--grad_scaler", action="store_true",
                   help="dynamic loss scaling as the reference's GradScaler (fused non-finite check, "
                        "skip + back-off on device); unnecessary for bf16, off by default")
    p.add_argument("--dropout", type=float, default=0.0)
    p.add_argument("--recompute", action="store_true",
                   help="activation recompute: keep only each layer's input, re-run its forward in backward")
    p.add_argument("--synthetic_data", action="store_true",
                   help="use the synthetic token corpus (default when HF data is unavailable)")
    p.add_argument("--data_path", type=str, default=None,
                   help="pre-tokenised flat token file (.bin) read by the native mmap loader")
    p.add_argument("--token_bytes", type=int, default=2, choices=[2, 4], help="bytes per token in --data_path")
    p.add_argument("--train_samples", type=int, default=20000, help="synthetic corpus size")
    p.add_argument("--val_samples", type=int, default=256)
    p.add_argument("--max_steps", type=int, default=0, help="stop each epoch after this many steps (0 = all)")
    p.add_argument("--eval_steps", type=int, default=0, help="limit validation batches (0 = all)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--resume", type=str, default=None, help="checkpoint file or 'latest'")
    p.add_argument("--checkpoint_dir", type=str, default="checkpoints")
    p.add_argument("--save_every", type=int, default=0,
                   help="also checkpoint (model + optimizer + RNG) every N optimizer steps")
    p.add_argument("--no_save", action="store_true")
    p.add_argument("--no_generate", action="store_true")
    p.add_argument("--bucket_mb", type=float, default=128.0, help="DDP gradient bucket size")
    p.add_argument("--reduce_dtype", type=str, default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--no_overlap", action="store_true", help="all-reduce after backward instead of during")
    p.add_argument("--comm", default=os.environ.get("DPC_COMM", "auto"), choices=["auto", "torch", "native", "ipc"],
                   help="collective transport of every engine (parallel/transport.py): the native C++ RCCL "
                        "communicator on its own HIP stream (auto = on a GPU), torch.distributed, or ipc -- "
                        "direct peer-access collectives over xGMI (parallel/ipc_comm.py; DDP / FSDP)")
    p.add_argument("--profile", type=str, default=None, help="write a torch.profiler trace here")
    p.add_argument("--log_jsonl", type=str, default=None, help="append step metrics as JSON lines")
    p.add_argument("--cpu", action="store_true", help="force CPU (gloo) even if a GPU is present")
    # --- debug switches
    p.add_argument("--serialize_kernels", action="store_true",
                   help="serialise every HIP launch / copy and synchronise after each native kernel, "
                        "so a faulting kernel is named at its launch (DPC_SERIALIZE=1)")
    p.add_argument("--stream_check", action="store_true",
                   help="assert that every asynchronous collective is waited on before the step ends and "
                        "poll RCCL for asynchronous errors (DPC_STREAM_CHECK=1)")
    p.add_argument("--coll_check", action="store_true",
                   help="all-gather a (sequence, op, shape, dtype) fingerprint before each collective and "
                        "raise on a mismatch across ranks (DPC_COLL_CHECK=1)")
    if recipe in ("pipe", "pipe_ddp"):
        p.add_argument("--pp_size", type=int, default=0, help="pipeline stages (0 = world size / dp)")
        p.add_argument("--num_microbatches", type=int, default=0, help="0 = 4 x stages (1 for a single stage)")
        p.add_argument("--schedule", type=str, default="1f1b", choices=["1f1b", "gpipe", "zb", "zb2"],
                       help="micro-batch schedule: 1F1B (PipeDream-flush), GPipe, or zero-bubble (1F1B with the "
                            "weight-gradient passes deferred into the pipeline bubbles; zb2: twice the forwards in "
                            "flight and every W deferrable -- less bubble, more HBM)")
        p.add_argument("--pp_comm_dtype", type=str, default="fp32", choices=["fp32", "bf16"],
                       help="wire format of the stage-boundary activations and their gradients")
    if recipe == "pipe_ddp":
        p.add_argument("--dp_size", type=int, default=0,
                       help="data-parallel replicas per stage (0 = world size / 2: PP = 2 x DP = N / 2)")
    if recipe == "fsdp":
        p.add_argument("--prefetch", type=int, default=1, help="units all-gathered ahead")
        p.add_argument("--no_reshard_after_forward", action="store_true")
    return p


def apply_preset(args) -> None:
    if getattr(args, "model", None):
        for k, v in PRESETS[args.model].items():
            if k == "activation" and args.activation is not None:
                continue
            setattr(args, k, v)
    if getattr(args, "activation", None) is None:
        args.activation = "relu"


def parse(recipe: str = "single", argv=None):
    args = build_parser(recipe).parse_args(argv)
    apply_preset(args)
    return args
