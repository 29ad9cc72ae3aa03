"""Recipe driver: the body of ``main-single.py`` / ``main-ddp.py`` / ``main-fsdp.py`` /
``main-pipe.py`` / ``main-pipe-ddp.py``.

Reference entrypoints: ``/root/reference/main-single.py:18-151`` (single device),
``main-ddp.py:38-187`` (DDP), ``main-fsdp.py:42-202`` (FSDP + CPU offload),
``main-pipe.py:85-221`` (GPipe), ``main-pipe-ddp.py:1`` (an empty stub in the reference;
implemented here as a PP x DP mesh).  All share flags (``config.py``), data, model and
the trainer; only the engine differs.
"""
from __future__ import annotations

import os

import torch

from .config import parse
from .engine.trainer import Trainer
from .models.gpt import TransformerDecoderLM
from .parallel import comm
from .utils.data import get_dataset, get_tokenizer, transform_dataset

PAD_ID = 2  # reference main-single.py:23


def build_model(args, vocab_size: int, device) -> TransformerDecoderLM:
    torch.manual_seed(args.seed)
    with torch.device(device):
        model = TransformerDecoderLM(
            dim=args.dim, head_dim=args.head_dim, heads=args.heads, num_layers=args.num_layers,
            vocab_size=vocab_size, max_position_embeddings=args.sequence_length,
            dropout=args.dropout, activation=args.activation,
        )
    model.recompute = bool(getattr(args, "recompute", False))
    return model


def pipe_mesh(recipe: str, world: int, pp_size: int = 0, dp_size: int = 0) -> tuple[int, int]:
    """(pp, dp) of the pipeline recipes: ``main-pipe.py`` is one pipeline over every rank;
    ``main-pipe-ddp.py`` defaults to the BASELINE.json hybrid, 2 stages x N / 2 replicas
    (8 ranks: pp2 x dp4)."""
    dp = dp_size or 1
    if recipe == "pipe_ddp" and not dp_size:
        pp0 = pp_size or 2
        dp = world // pp0 if world % pp0 == 0 else 1
    pp = pp_size or max(1, world // dp)
    return pp, dp


def build_engine(recipe: str, model, info, args, force_dist: bool = False):
    """``force_dist``: at one rank, take the engines' N > 1 code path over a native 1-rank RCCL
    communicator (bucketed DDP store, sharded FSDP store, replica DDP store of the pipeline) --
    bench.py --force_dist_path profiles it on one GPU."""
    compute_dtype = torch.float32 if args.disable_amp else None
    # --reduce_dtype: the wire/reduction dtype of the gradient collectives of every recipe (DDP
    # bucket all-reduce, FSDP reduce-scatter, the PP x DP replica all-reduce); the reference
    # reduces fp32 (autocast keeps fp32 grads, /root/reference/main-fsdp.py:64-69)
    reduce_dtype = torch.bfloat16 if getattr(args, "reduce_dtype", "fp32") == "bf16" else torch.float32
    comm_kind = "native" if force_dist else getattr(args, "comm", "auto")
    # the cookbook's "compile": capture the whole step into a HIP graph (dropout included: the
    # per-forward seed is a device counter the mask kernels read, so replays draw fresh masks --
    # models/gpt.py:next_dropout_seed).  On every rank, as the reference compiles on every rank
    # (/root/reference/main-ddp.py:60-61): the capture is collective -- a barrier before it, and
    # every rank graphs or none does (engine/base.py:GraphedStep) -- and the RCCL calls inside it
    # are the native communicator's, captured at one rank by tests/test_native_comm.py.
    # --disable_compile keeps eager steps (bench.py's N > 1 runs do: same speed, measured at N = 1);
    # never under --coll_check, whose fingerprints are host-synchronous collectives
    graph = (not args.disable_compile and not args.disable_amp
             and not getattr(args, "coll_check", False))
    if recipe in ("single", "ddp"):
        from .engine.data_parallel import DataParallelEngine

        return DataParallelEngine(
            model, info.device, lr=args.learning_rate, bucket_mb=args.bucket_mb,
            reduce_dtype=reduce_dtype,
            overlap=not args.no_overlap, compute_dtype=compute_dtype, graph=graph,
            comm_kind=comm_kind, grad_scaler=getattr(args, "grad_scaler", False), force_ddp_store=force_dist,
        )
    if recipe == "fsdp":
        from .engine.fsdp import FSDPEngine

        return FSDPEngine(model, info.device, lr=args.learning_rate, prefetch=args.prefetch,
                          reshard_after_forward=not args.no_reshard_after_forward,
                          cpu_offload=args.cpu_offload, compute_dtype=compute_dtype,
                          reduce_dtype=reduce_dtype, grad_scaler=getattr(args, "grad_scaler", False), graph=graph, comm_kind=comm_kind,
                          force_sharded=force_dist)
    if recipe in ("pipe", "pipe_ddp"):
        from .engine.pipeline import PipelineEngine

        pp, dp = pipe_mesh(recipe, info.world_size, args.pp_size, getattr(args, "dp_size", 0))
        wire = {"fp32": None, "bf16": torch.bfloat16}[getattr(args, "pp_comm_dtype", "fp32")]
        return PipelineEngine(model, info.device, lr=args.learning_rate, pp=pp, dp=dp,
                              num_microbatches=args.num_microbatches,
                              schedule=args.schedule, bucket_mb=args.bucket_mb,
                              compute_dtype=compute_dtype, grad_scaler=getattr(args, "grad_scaler", False),
                              comm_kind=comm_kind, wire_dtype=wire, graph=graph, force_dist=force_dist,
                              reduce_dtype=reduce_dtype)
    raise ValueError(recipe)


def apply_debug_switches(args) -> None:
    """SURVEY.md §5.2 switches: serialised launches, stream-order checks, collective
    fingerprints."""
    if getattr(args, "serialize_kernels", False):
        from .ops import _lib

        _lib.enable_serialize()
    if getattr(args, "stream_check", False):
        from .parallel import transport

        transport.set_stream_check(True)
    if getattr(args, "coll_check", False):
        comm.set_coll_check(True)


def run(recipe: str, argv=None):
    args = parse("pipe_ddp" if recipe == "pipe_ddp" else recipe, argv)
    apply_debug_switches(args)  # before the HIP runtime starts (init_dist binds the device)
    info = comm.init_dist(force_cpu=args.cpu)
    if recipe == "single" and info.world_size > 1:
        raise SystemExit("main-single.py runs one process; use main-ddp.py under torchrun")
    if info.is_main:
        print(f"[{recipe}] world={info.world_size} device={info.device} backend={info.backend}")
    synthetic = True if args.synthetic_data else None
    tokenizer = get_tokenizer(max_length=args.sequence_length, offline_stub=synthetic)
    tokenizer.pad_token_id = PAD_ID
    model = build_model(args, tokenizer.vocab_size, info.device)
    model.dropout_seed_base = args.seed * 65537 + info.rank  # distinct masks per rank
    engine = build_engine(recipe, model, info, args)
    train, val = get_dataset(slice_size=args.dataset_slice, synthetic=synthetic,
                             seq_len=args.sequence_length, n_train=args.train_samples,
                             n_val=args.val_samples, seed=args.seed)
    train = transform_dataset(train, tokenizer, max_length=args.sequence_length, num_proc=args.num_workers)
    val = transform_dataset(val, tokenizer, max_length=args.sequence_length, num_proc=args.num_workers)
    trainer = Trainer(args, engine, tokenizer, PAD_ID)
    try:
        path = trainer.fit(train, val)
    finally:
        comm.cleanup_dist()
    return trainer, path
